#!/usr/bin/env python3
"""bench.py - frames/s stacked (4096x4096 u16, sigma-clip) + achieved HBM GB/s on MI355X.

BASELINE.json metric, measured on BASELINE.json configs[2] (the configuration the metric
is quoted on that fits one GPU): sigma-clip rejection stack (SIGMA, sig = (4, 3),
NO_NORM, registration shifts applied) of 512 synthetic 4096x4096 u16 mono frames,
frames resident in HBM (generated on the device by include/sg_synth.h).

One step = one sg_stack_u16_device() call over the whole 512-frame sequence.
Multi-GPU (torchrun, one process per GPU): weak scaling by row bands -- one sequence of
512 frames of (4096*G) x 4096 with one set of registration shifts; rank r owns output rows
[4096 r, 4096 (r+1)) and holds only the frame rows they read (its band plus the rows the
shifts reach, sg_stack_desc.resident_rows); no data-path collective (each rank's band is
written to its own output); the 6 rejection counters and the step times are all-reduced
(max for time).

Output: one JSON line on rank 0 (see README / DESIGN.md for the fields).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=["sigma", "register-mean", "winsorized-rgb"], default="sigma",
                    help="sigma = BASELINE configs[2] (the metric's configuration, default); "
                         "register-mean = configs[1]; winsorized-rgb = configs[4] at one GPU")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--height", type=int, default=4096)
    ap.add_argument("--rejection", default="sigma")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--normalize", choices=["none", "additive-scaling", "multiplicative-scaling"], default="none",
                    help="sigma workload: per-frame normalisation (synthetic location / scale, as "
                         "compute_normalization derives them)")
    ap.add_argument("--maxshift", type=int, default=16, help="synthetic registration shift range")
    ap.add_argument("--even-shifts", action="store_true",
                    help="A/B only: round x shifts down to even (4-byte aligned pixel-pair loads)")
    ap.add_argument("--zero-shift", choices=["x", "y"], default=None,
                    help="A/B only: drop the x or y registration shifts")
    ap.add_argument("--frame-pad", type=int, default=0,
                    help="extra elements between frames in HBM (breaks power-of-two frame strides)")
    ap.add_argument("--cpu-rows", type=int, default=1024, help="rows of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="OpenMP threads of the CPU baseline (the GPU box's CPU share is 16)")
    return ap.parse_args()


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def synth_shifts_np(N, seed, maxshift):
    """registration shifts of the synthetic sequence (include/sg_synth.h sg_synth_shift):
    (shiftx, shifty) = (-dx_f, -dy_f), frame 0 = 0"""
    import numpy as np
    shx = np.zeros(N, dtype=np.int32)
    shy = np.zeros(N, dtype=np.int32)
    for f in range(1, N):
        h = _mix64(seed ^ 0x51B1 ^ (f << 32))
        if maxshift > 0:
            span = 2 * maxshift + 1
            shx[f] = -((h & 0xFFFFFFFF) % span - maxshift)
            shy[f] = -(((h >> 32) & 0xFFFFFFFF) % span - maxshift)
    return shx, shy


def cpu_baseline(args, N, W):
    """Oracle (C restatement of the reference stacker, -O2 -fopenmp, the reference's block
    partition and OpenMP schedule) on a bounded sample of the same workload."""
    import numpy as np
    import oracle_lib as orc
    rows = min(args.cpu_rows, args.height)
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    lib = orc.load()
    try:
        import ctypes
        ctypes.CDLL("libgomp.so.1").omp_set_num_threads(threads)
    except OSError:
        pass
    # the same synthetic scene and registration shifts as the GPU run, rows [0, rows)
    frames = orc.synth(N, 1, rows, W, seed=0x5151, maxshift=16)
    sx, sy = orc.synth_shifts(N, seed=0x5151, maxshift=16)
    t0 = time.perf_counter()
    rc, out, rej = orc.stack_rejection(frames, 2, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                       max_thread=threads, max_number_of_rows=rows)
    dt = time.perf_counter() - t0
    del frames
    frac = rows / args.height
    return {"value": round(N * frac / dt, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"oracle stack_mean_with_rejection SIGMA(4,3), {N} frames x {rows} rows x {W} "
                      f"cols ({threads} OpenMP threads); frames/s scaled by {rows}/{args.height} rows",
            "seconds": round(dt, 3), "rc": rc}


def roofline(achieved, algo_bytes, N, H, W, rejection):
    """roofline object of the dominant kernel (k_stack_hist for sigma): achieved = algorithmic
    bytes per launch / HIP-event kernel time; traffic = HBM bytes per launch from the
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the same workload (scripts/gpu_pmc_traffic.sh
    -> profiles/traffic_<workload>.json, corrected per MI355X_MICROARCH.md), when present"""
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None}
    path = os.path.join(ROOT, "profiles", f"traffic_{rejection}_{N}x{H}x{W}.json")
    if os.path.exists(path):
        with open(path) as f:
            t = json.load(f)
        r["traffic"] = int(t["traffic_bytes"])
        r["traffic_unit"] = "B/launch"
        r["traffic_over_algorithmic"] = round(t["traffic_bytes"] / algo_bytes, 4)
        r["traffic_src"] = os.path.relpath(path, ROOT)
    return r


def main_config(args):
    """BASELINE configs[1] (register-mean: DFT registration of 128 full 2048x2048 SER-like
    frames + NO_REJEC mean stack with the found shifts) and configs[4] (winsorized-rgb: 256
    3-plane 6000x4000 frames, DFT registration of a centred 2048x2048 selection of layer 1,
    WINSORIZED (4, 3) stack), one GPU, frames resident in HBM.  One step = registration +
    stack; the stage times are reported beside the step time."""
    import numpy as np
    import torch
    import sirilgpu as sg
    torch.cuda.set_device(0)
    ctx = sg.Context([0])
    if args.workload == "register-mean":
        N, C, H, W, S, layer, rej, cfg = 128, 1, 2048, 2048, 2048, 0, sg.NO_REJEC, "BASELINE configs[1]"
    else:
        N, C, H, W, S, layer, rej, cfg = 256, 3, 4000, 6000, 2048, 1, sg.WINSORIZED, "BASELINE configs[4], 1 GPU"
    fstride = C * H * W
    frames = torch.empty(N * fstride, dtype=torch.int16, device="cuda")
    out = torch.empty(C * H * W, dtype=torch.int16, device="cuda")
    ctx.synth_fill(frames.data_ptr(), N, C, H, W, 0, H, 0x5EED, 16)
    fv = frames.view(N, C, H, W)
    y0, x0 = (H - S) // 2, (W - S) // 2

    def step():
        t0 = time.perf_counter()
        if S == H and S == W and C == 1:
            sel = frames                      # full-frame selection: the frames themselves
        else:                                 # seq_read_frame_part of layer `layer`
            sel = fv[:, layer, y0:y0 + S, x0:x0 + S].contiguous()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sx, sy, q = ctx.register_dft_device(sel.data_ptr(), N, S)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=rej, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                  max_thread=8, max_number_of_rows=H)
        rejc, _ = ctx.stack_device(desc, frames.data_ptr(), fstride, H * W, out.data_ptr(), 0, H)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        return (t1 - t0, t2 - t1, t3 - t2), ctx.stats(), sx, sy

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stages = np.zeros(3)
    kms = []
    for _ in range(args.steps):
        st, stats, sx, sy = step()
        stages += np.array(st)
        kms.append(stats.kernel_ms)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    stages /= args.steps
    # registration shifts must recover the synthetic translations (frame 0 = reference)
    ex, ey = synth_shifts_np(N, 0x5EED, 16)
    reg_ok = bool(np.array_equal(sx, ex) and np.array_equal(sy, ey))
    kavg = sum(kms) / len(kms)
    stack_bytes = N * C * H * W * 2 + C * H * W * 2
    achieved = stack_bytes / (kavg * 1e-3) / 1e9
    reg_bytes = N * S * S * 58          # stated 2-pass c64 FFT model, SURVEY.md section 8(d)
    res = {
        "metric": "frames/sec stacked (registration + stack) + achieved HBM GB/s",
        "value": round(N / (elapsed / args.steps), 2), "unit": "frames/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u16",
        "data": "synthetic (include/sg_synth.h, generated in HBM)",
        "config": {"workload": f"{args.workload} {N}x{C}x{H}x{W} ({cfg})", "frames": N, "layers": C,
                   "height": H, "width": W, "selection": S, "register_layer": layer,
                   "rejection": "none" if rej == sg.NO_REJEC else "winsorized"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": "stack"},
        "stage_ms": {"selection": round(stages[0] * 1e3, 3), "register": round(stages[1] * 1e3, 3),
                     "stack": round(stages[2] * 1e3, 3), "stack_kernel": round(kavg, 3)},
        "register_GBps_model": round(reg_bytes / stages[1] / 1e9, 1),
        "slow_pixels": int(stats.slow_pixels), "redo_pixels": int(stats.chain_pixels),
        "register_shifts_exact": reg_ok,
    }
    print(json.dumps(res), flush=True)
    ctx.close()


def main():
    args = parse()
    if args.workload != "sigma":
        return main_config(args)
    import numpy as np
    import torch
    import sirilgpu as sg

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # SG_BENCH_REHEARSE=1 (testing only): every rank on cuda:0 over gloo, to rehearse the
        # multi-rank flow on a one-GPU box; the driver's runs use one GPU per rank over RCCL
        rehearse = os.environ.get("SG_BENCH_REHEARSE") == "1"
        torch.cuda.set_device(0 if rehearse else local)
        dist.init_process_group("gloo" if rehearse else "nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    N, W, H = args.frames, args.width, args.height
    rej_mode = {"sigma": sg.SIGMA, "winsorized": sg.WINSORIZED, "none": sg.NO_REJEC,
                "percentile": sg.PERCENTILE}[args.rejection]
    ctx = sg.Context([dev])
    # one sequence of N frames of (H*world) x W; this rank owns output rows [rank*H,
    # (rank+1)*H) and holds only the frame rows they read (the band plus the rows its
    # registration shifts reach), addressed through a biased base pointer
    Htot = H * world
    shx, shy = synth_shifts_np(N, 0x5151, args.maxshift)
    if args.even_shifts:
        shx &= ~1
    if args.zero_shift:
        (shx if args.zero_shift == "x" else shy)[:] = 0
    b, e = rank * H, (rank + 1) * H
    lo, hi = max(0, b - int(shy.max())), min(Htot - 1, e - 1 - int(shy.min()))
    nres = hi - lo + 1
    fstride = nres * W + args.frame_pad
    frames = torch.empty(N * fstride, dtype=torch.int16, device="cuda")
    out = torch.empty(Htot * W, dtype=torch.int16, device="cuda")
    base = frames.data_ptr() - lo * W * 2
    ctx.synth_fill(base, N, 1, Htot, W, lo, hi + 1, 0x5151, args.maxshift, frame_stride=fstride)
    norm_mode, off, mul, scale = sg.NO_NORM, None, None, None
    if args.normalize != "none":
        # synthetic per-frame location / scale (the cached IKSS statistics), coefficients as
        # compute_normalization (src/stacking/stacking.c:79-190) forms them, reference frame 0
        # (the synthetic frames share one background, so their statistics differ only by noise)
        i = np.arange(N, dtype=np.float64)
        loc = 1000.0 + 0.6 * np.sin(0.37 * i)
        scl = 30.0 + 0.3 * np.cos(0.23 * i)
        if args.normalize == "additive-scaling":
            norm_mode = sg.ADDITIVE_SCALING
            scale = scl[0] / scl
            off = scale * loc - loc[0]
        else:
            norm_mode = sg.MULTIPLICATIVE_SCALING
            scale = scl[0] / scl
            mul = loc[0] / loc
    desc, keep = sg.make_desc(sg.MEAN, N, W, Htot, 1, rejection=rej_mode, sig=(4.0, 3.0),
                              shiftx=shx, shifty=shy, normalize=norm_mode, offset=off, mul=mul, scale=scale,
                              max_thread=8, max_number_of_rows=Htot, resident_rows=(lo, hi + 1))

    def step():
        return ctx.stack_device(desc, base, fstride, nres * W, out.data_ptr(), b, e)

    for _ in range(args.warmup):
        step()
    kms, slow, redo = [], 0, 0
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rej_tot = None
    for _ in range(args.steps):
        rej, _ = step()
        st = ctx.stats()
        kms.append(st.kernel_ms)
        slow = st.slow_pixels
        redo = st.chain_pixels
        rej_tot = rej
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        import sirilgpu_dist as sd
        cdev = "cpu" if os.environ.get("SG_BENCH_REHEARSE") == "1" else "cuda"
        elapsed = sd.max_time(elapsed, dist, device=cdev)
        rej_tot = sd.sum_counters(rej_tot, dist, device=cdev)
    ms_step = elapsed / args.steps * 1e3
    frames_per_s = N * world / (elapsed / args.steps)
    kavg = sum(kms) / len(kms)
    algo_bytes = N * H * W * 2 + H * W * 2
    achieved = algo_bytes / (kavg * 1e-3) / 1e9
    if rank == 0:
        res = {
            "metric": "frames/sec stacked (4096x4096 u16, sigma-clip) + achieved HBM GB/s",
            "value": round(frames_per_s, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (include/sg_synth.h, generated in HBM)",
            "config": {"workload": f"sigma-clip stack {N}x{H}x{W} u16 mono per GPU (BASELINE configs[2]"
                                   + (")" if world == 1 else f"; one {N}x{Htot}x{W} sequence in {world} row bands)"),
                       "frames": N, "height": H, "width": W, "rejection": args.rejection,
                       "sig": [4.0, 3.0], "normalize": args.normalize, "parallelism": f"row-band x{world}"},
            "roofline": roofline(achieved, algo_bytes, N, H, W, args.rejection
                                 if args.normalize == "none" else f"{args.rejection}_{args.normalize}"),
            "kernel_ms": round(kavg, 3),
            "slow_pixels": int(slow),
            "redo_pixels": int(redo),
            "rejected": [int(x) for x in rej_tot.reshape(-1)[:2]],
        }
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(args, N, W)
        print(json.dumps(res), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
