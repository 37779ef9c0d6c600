#!/usr/bin/env python3
"""bench.py - frames/s stacked (4096x4096 u16, sigma-clip) + achieved HBM GB/s on MI355X.

BASELINE.json metric.  Workloads (frames synthetic, include/sg_synth.h, generated in HBM):
  sigma (default)  configs[2] at one GPU: SIGMA (4, 3) stack of 512 x 4096 x 4096 u16 mono with
                   registration shifts.  At N GPUs (torchrun, one process per GPU) the stack
                   partitions into row bands (the reference's own block partition,
                   stacking.c:1397-1476, lifted to GPUs), so by default (WEAK scaling, no
                   data-path collective) each rank stacks a full 4096-row band of one 512-frame
                   (4096 N)-row sequence, holding only its band + the rows its shifts reach; the
                   rejection counters are summed after the timed region.  --scaling strong:
                   configs[3] as a fixed job, the one 4096-row sequence split into N bands of
                   4096/N rows, the output bands gathered to rank 0 over RCCL inside the timed
                   region with the counters all-reduced.
  register-mean    configs[1]: DFT registration of 128 full 2048 x 2048 frames + NO_REJEC mean.
  winsorized-rgb   configs[4]: 256 x 3 x 4000 x 6000, DFT registration of layer 1's centred 2048
                   selection + WINSORIZED (4, 3).  At N GPUs: registration sharded over frames (each
                   rank its block + the reference, shifts all-gathered, normalizeQualityData over all
                   frames), the stack over row bands, output gathered to rank 0.
  median           stack_median of the configs[2] frames (512 x 4096 x 4096 u16, registration ignored as
                   the reference's :703-722 does): the histogram rank path (k_stack_hist<8>).
  sum-fits         configs[0]: stack_summing of 16 x 1024 x 1024 u16 FITS files, end to end from the
                   files (host-pull path: reads + PCIe + kernels), the CPU reference configuration.

One step = one pass of the workload.  Rank 0 prints ONE JSON line (fields: README / DESIGN.md).
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
    ap.add_argument("--workload", choices=["sigma", "median", "register-mean", "winsorized-rgb", "sum-fits",
                                           "register-mean-file"],
                    default="sigma",
                    help="sigma = BASELINE configs[2] (1 GPU) / configs[3] (N GPUs, default); register-mean = "
                         "configs[1]; winsorized-rgb = configs[4]; sum-fits = configs[0]")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="weak",
                    help="sigma at N GPUs: strong = one 4096-row sequence in N bands + gather (configs[3]); "
                         "weak = a 4096-row band per GPU")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--height", type=int, default=4096)
    ap.add_argument("--rejection", default="sigma")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--normalize", choices=["none", "additive", "additive-scaling", "multiplicative-scaling"], default="none",
                    help="sigma workload: per-frame normalisation (synthetic location / scale, as "
                         "compute_normalization derives them)")
    ap.add_argument("--band-of", type=int, default=0,
                    help="A/B at 1 GPU: stack only band 0 of the configs[3] job split into this many row bands "
                         "(one rank's call of the strong form), only that band's rows resident")
    ap.add_argument("--strong-gather", choices=["overlap", "serial", "none"], default="overlap",
                    help="strong form (and --band-of): overlap = band calls with their tails on the library's "
                         "tail stream, output bands gathered on a comm stream from two alternating buffers; "
                         "serial = tail and gather on the call's stream; none = no gather")
    ap.add_argument("--stack-stream", choices=["side", "call"], default="call",
                    help="register-mean / winsorized-rgb at 1 GPU: call = each step's stack queued on the "
                         "registration's stream (default); side = on a second stream, beside the next step's "
                         "registration (A/B: configs[1] 3.26 -> 3.20 ms per step, configs[4] 33.3 -> 33.6 ms, and "
                         "the registration's device span then includes the stack it shares the chip with)")
    ap.add_argument("--maxshift", type=int, default=16, help="synthetic registration shift range")
    ap.add_argument("--even-shifts", action="store_true",
                    help="A/B only: round x shifts down to even (4-byte aligned pixel-pair loads)")
    ap.add_argument("--zero-shift", choices=["x", "y"], default=None,
                    help="A/B only: drop the x or y registration shifts")
    ap.add_argument("--frame-pad", type=int, default=0,
                    help="extra elements between frames in HBM (breaks power-of-two frame strides)")
    ap.add_argument("--selection", type=int, default=0,
                    help="register-mean / winsorized-rgb: side of the registration selection (default 2048; "
                         "e.g. 4000 = configs[4]'s full height, a non-power-of-two side)")
    ap.add_argument("--cpu-rows", type=int, default=1024, help="rows of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="OpenMP threads of the CPU baseline (default: the CPUs this process may run on, "
                         "sched_getaffinity, capped by the cgroup's cpu.max quota)")
    return ap.parse_args()


def cpu_share():
    """the CPUs this process may use: its affinity mask, capped by the cgroup v2 cpu.max quota (CPUs'
    worth of time per period) when one is set and by OMP_NUM_THREADS when the host sets one (the
    GPU box exports its per-GPU CPU share there); the CPU baseline runs that many OpenMP threads,
    as the reference's team is com.max_thread = omp_get_num_procs() (src/main.c:375)"""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    raw = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            raw = f.read().strip()
        q, per = raw.split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        use = min(use, int(omp))
    return {"affinity_cpus": aff, "cgroup_cpu_max": raw, "cgroup_quota_cpus": quota, "omp_num_threads": omp,
            "os_cpu_count": os.cpu_count(), "threads": use}


def cpu_threads(args):
    return args.cpu_threads if args.cpu_threads > 0 else cpu_share()["threads"]


def self_launch(args):
    """--gpus N > 1 without a launcher: start N ranks as fresh child processes (torch.distributed.run,
    one process per GPU, rendezvous on 127.0.0.1) before anything here touches a GPU, and exit with
    their return code.  Under a launcher, WORLD_SIZE must equal --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}", file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


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


def cpu_model():
    """the host CPU's model name (lscpu's 'Model name', from /proc/cpuinfo)"""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _omp_threads(n):
    import ctypes
    try:
        ctypes.CDLL("libgomp.so.1").omp_set_num_threads(n)
    except OSError:
        pass


def cpu_baseline(args, N, W, median=False):
    """configs[2]: the oracle (C restatement of stack_mean_with_rejection / stack_median, -O2
    -fopenmp, the reference's block partition and OpenMP schedule) on a bounded sample of the
    same workload"""
    import oracle_lib as orc
    rows = min(args.cpu_rows, args.height)
    threads = cpu_threads(args)
    orc.load()
    _omp_threads(threads)
    frames = orc.synth(N, 1, rows, W, seed=0x5151, maxshift=16)
    sx, sy = orc.synth_shifts(N, seed=0x5151, maxshift=16)
    t0 = time.perf_counter()
    if median:
        rc, out = orc.stack_median(frames, max_thread=threads, max_number_of_rows=rows)
        what = "stack_median"
    else:
        rej_mode = {"sigma": 2, "winsorized": 4, "none": 0, "percentile": 1, "sigmedian": 3,
                    "linearfit": 5}[args.rejection]
        rc, out, rej = orc.stack_rejection(frames, rej_mode, sig=(4.0, 3.0) if rej_mode != 1 else (0.2, 0.1),
                                           shiftx=sx, shifty=sy, max_thread=threads, max_number_of_rows=rows)
        what = f"stack_mean_with_rejection {args.rejection}"
    dt = time.perf_counter() - t0
    del frames
    frac = rows / args.height
    return {"value": round(N * frac / dt, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "cpu_share": cpu_share(),
            "sample": f"oracle {what}, {N} frames x {rows} rows x {W} cols ({threads} OpenMP threads), "
                      f"timed on {rows} of {args.height} rows; frames/s = {N} x {rows}/{args.height} / seconds",
            "seconds": round(dt, 3), "rc": rc}


def cpu_baseline_config(args, workload, N, C, H, W, S, layer):
    """configs[1] / configs[4]: the oracle's register_shift_dft over 32 frames with the reference's
    OpenMP loop over frames (registration.c:276-279) on the process's CPU share (cpu_share), timed,
    and its stacker (NO_REJEC mean / WINSORIZED, same threads) on a row sample; the step estimate is
    N x (registration seconds per frame) + t_stack scaled to the full image.  The oracle's FFT is
    a plain radix-2 complex-double transform, not FFTW (FFTW_ESTIMATE plans are several times
    faster per transform), which the sample text states"""
    import oracle_lib as orc
    threads = cpu_threads(args)
    orc.load()
    _omp_threads(threads)
    nreg = 33
    y0, x0 = (H - S) // 2, (W - S) // 2
    sel = orc.synth_window(nreg, layer, y0, x0, S, S, seed=0x5EED, maxshift=16)
    t0 = time.perf_counter()
    orc.register_dft(sel)                 # the reference's spectrum + (nreg - 1) registered frames
    t_reg = (time.perf_counter() - t0) / (nreg - 1)
    del sel
    rows = min(64 if workload == "winsorized-rgb" else 256, H)
    frames = orc.synth(N, C, rows, W, seed=0x5EED, maxshift=16)
    sx, sy = orc.synth_shifts(N, seed=0x5EED, maxshift=16)
    rej = 4 if workload == "winsorized-rgb" else 0
    t0 = time.perf_counter()
    orc.stack_rejection(frames, rej, sig=(4.0, 3.0), shiftx=sx, shifty=sy, max_thread=threads, max_number_of_rows=rows)
    t_stack = (time.perf_counter() - t0) * H / rows
    del frames
    step = N * t_reg + t_stack
    return {"value": round(N / step, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "cpu_share": cpu_share(),
            "sample": f"oracle register_shift_dft on {nreg - 1} frames of {S}^2 + the reference, {threads} OpenMP "
                      f"threads over frames as :276-279 (measured {t_reg * 1e3:.1f} ms per frame; its FFT is a plain "
                      f"radix-2 complex-double transform, not FFTW) + oracle "
                      f"{'WINSORIZED' if rej else 'NO_REJEC mean'} on {rows} of {H} rows x {C} channels "
                      f"({threads} threads), stack time scaled by {H}/{rows}",
            "seconds_register_per_frame": round(t_reg, 4), "seconds_stack_scaled": round(t_stack, 3)}


def load_traffic(path, r, key="traffic_bytes"):
    """the PMC capture at `path` (scripts/pmc_traffic.py) when it describes the kernel sources
    being run: its src_id must equal the digest of the current sources (sg_srcid); a capture of
    an older build (or one without an id) is reported as traffic_stale and its bytes dropped"""
    import sg_srcid
    if not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    kern = ",".join(t["kernels"]) if "kernels" in t else t["kernel"]
    try:
        now = sg_srcid.source_id(kern)
    except (KeyError, OSError):
        now = None
    if t.get("src_id") is None or t.get("src_id") != now:
        r["traffic_stale"] = {"src": os.path.relpath(path, ROOT), "capture_src_id": t.get("src_id"),
                              "built_src_id": now}
        return None
    r["traffic_src"] = os.path.relpath(path, ROOT)
    r["traffic_src_id"] = now
    return t


def roofline(achieved, algo_bytes, N, H, W, rejection, with_traffic=True, profiles=None):
    """roofline object of the dominant kernel (k_stack_hist for sigma): achieved = algorithmic
    bytes per launch / HIP-event kernel time; traffic = HBM bytes per launch from the
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the same workload (scripts/gpu.sh pmc ->
    profiles/traffic_<workload>.json, corrected per MI355X_MICROARCH.md), when present and
    captured from the sources being run (load_traffic)"""
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None}
    path = os.path.join(profiles or os.path.join(ROOT, "profiles"), f"traffic_{rejection}_{N}x{H}x{W}.json")
    t = load_traffic(path, r) if with_traffic else None
    if t is not None:
        r["traffic"] = int(t["traffic_bytes"])
        r["traffic_unit"] = "B/launch"
        r["traffic_over_algorithmic"] = round(t["traffic_bytes"] / algo_bytes, 4)
    return r


class Dist:
    """one process per GPU (torchrun): RCCL ("nccl") on the node; SG_BENCH_REHEARSE=1 (testing
    only) runs every rank on cuda:0 over gloo with CPU staging of the collectives"""

    def __init__(self):
        import torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        self.rehearse = os.environ.get("SG_BENCH_REHEARSE") == "1"
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(0 if self.rehearse else local)
            dist.init_process_group("gloo" if self.rehearse else "nccl")
            self.dist = dist
        else:
            torch.cuda.set_device(0)
        self.cdev = "cpu" if self.rehearse else "cuda"

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max_time(self, t):
        import sirilgpu_dist as sd
        return sd.max_time(t, self.dist, device=self.cdev) if self.dist else t

    def gather_to_root(self, band, out_list):
        """rank 0 receives every rank's equal-sized band tensor (RCCL gather: each peer sends its
        band straight to rank 0 over its own xGMI link)"""
        # neither gloo nor RCCL has a 16-bit unsigned type: the bands travel as their bytes
        import torch
        as_bytes = lambda t: t.contiguous().view(torch.uint8)
        if self.rehearse:
            b = as_bytes(band.cpu())
            lst = [torch.empty_like(b) for _ in range(self.world)] if self.rank == 0 else None
            self.dist.gather(b, gather_list=lst, dst=0)
            if self.rank == 0:
                for o, t in zip(out_list, lst):
                    as_bytes(o).copy_(t)
        else:
            self.dist.gather(as_bytes(band), gather_list=[as_bytes(o) for o in out_list] if self.rank == 0 else None,
                             dst=0)

    def sum_counters(self, rej):
        import numpy as np
        import torch
        t = torch.as_tensor(np.asarray(rej, dtype=np.int64).reshape(-1), device=self.cdev)
        self.dist.all_reduce(t)
        return t

    def all_floats(self, x):
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.cdev)
        if not self.dist:
            return [float(x)]
        outs = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t)
        return [float(o.item()) for o in outs]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def timed(steps, warmup, step, D, after_warmup=None):
    import torch
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if after_warmup:
        after_warmup()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    return D.max_time(time.perf_counter() - t0)


def sigma_form(args, ctx, D, strong, gather_mode):
    """set up and time one form of the sigma / median workload on this rank; returns its numbers.
    strong: one sequence of N frames of H x W in `world` row bands; weak: one sequence of N frames
    of (H*world) x W, a full H-row band per rank.  Each rank holds only the frame rows its band
    reads (band + shift halo), addressed through a biased base pointer.  --band-of K at 1 GPU:
    rank 0's band of the strong form at K ranks, alone.  gather_mode (strong form): "overlap" = the
    band calls queued with SG_STACK_RESULT_AT_COLLECT and their output bands gathered to rank 0 on
    a comm stream from two alternating buffers (sirilgpu_dist.BandGatherPipeline), "serial" = the
    call's tail and the gather on the call's stream, "none" = no gather (at 1 GPU with --band-of the
    gather is a same-size device copy standing in for it)"""
    import numpy as np
    import torch
    import sirilgpu as sg
    import sirilgpu_dist as sd
    world, rank = D.world, D.rank
    N, W, H = args.frames, args.width, args.height
    rej_mode = {"sigma": sg.SIGMA, "winsorized": sg.WINSORIZED, "none": sg.NO_REJEC,
                "percentile": sg.PERCENTILE, "sigmedian": sg.SIGMEDIAN, "linearfit": sg.LINEARFIT}[args.rejection]
    median = args.workload == "median"
    method = sg.MEDIAN if median else sg.MEAN
    sig = (0.2, 0.1) if rej_mode == sg.PERCENTILE else (4.0, 3.0)
    nb = world if world > 1 else max(1, args.band_of)
    strong = strong or world == 1
    Htot = H if strong else H * world
    shx, shy = synth_shifts_np(N, 0x5151, args.maxshift)
    if args.even_shifts:
        shx &= ~1
    if args.zero_shift:
        (shx if args.zero_shift == "x" else shy)[:] = 0
    b, e = sd.row_band(rank, nb, H) if strong else (rank * H, (rank + 1) * H)
    if median:      # stack_median ignores the registration shifts (:703-722): the band's own rows
        lo, hi = b, e - 1
    else:
        lo, hi = max(0, b - int(shy.max())), min(Htot - 1, e - 1 - int(shy.min()))
    nres = hi - lo + 1
    fstride = nres * W + args.frame_pad
    frames = torch.empty(N * fstride, dtype=torch.int16, device="cuda")
    base = frames.data_ptr() - lo * W * 2
    ctx.synth_fill(base, N, 1, Htot, W, lo, hi + 1, 0x5151, args.maxshift, frame_stride=fstride)
    hband = -(-H // nb) if strong else H
    gathering = strong and nb > 1 and gather_mode != "none"
    norm_mode, off, mul, scale = sg.NO_NORM, None, None, None
    if args.normalize != "none":
        # synthetic per-frame location / scale (the cached IKSS statistics), coefficients as
        # compute_normalization (src/stacking/stacking.c:79-190) forms them, reference frame 0
        i = np.arange(N, dtype=np.float64)
        loc = 1000.0 + 0.6 * np.sin(0.37 * i)
        scl = 30.0 + 0.3 * np.cos(0.23 * i)
        scale = scl[0] / scl
        if args.normalize == "additive":
            norm_mode = sg.ADDITIVE
            scale = np.ones(N)
            off = loc - loc[0]
        elif args.normalize == "additive-scaling":
            norm_mode = sg.ADDITIVE_SCALING
            off = scale * loc - loc[0]
        else:
            norm_mode = sg.MULTIPLICATIVE_SCALING
            mul = loc[0] / loc
    flags = 0 if gathering and gather_mode == "serial" else sg.RESULT_AT_COLLECT
    desc, keep = sg.make_desc(method, N, W, Htot, 1, rejection=rej_mode if not median else sg.NO_REJEC, sig=sig,
                              shiftx=shx, shifty=shy, normalize=norm_mode, offset=off, mul=mul, scale=scale,
                              max_thread=8, max_number_of_rows=Htot, resident_rows=(lo, hi + 1), flags=flags)
    kms = []
    # the band calls, the serial gather and the pipeline's waits on one explicit stream (handle 0,
    # torch's default stream, would mean the library's own stream to sg_stack_u16_device_async)
    stream_obj = torch.cuda.Stream()
    prev_stream = torch.cuda.current_stream()
    torch.cuda.set_stream(stream_obj)
    stream = stream_obj.cuda_stream
    mk = lambda: torch.zeros(hband * W, dtype=torch.int16, device="cuda")

    if world > 1:
        gather_fn = lambda band, lst: D.gather_to_root(band, lst)
    else:       # --band-of K at 1 GPU: a device copy of the band standing in for the RCCL gather
        gather_fn = lambda band, lst: lst[0].copy_(band)
    if gathering and gather_mode == "overlap":
        comm = torch.cuda.Stream()
        pipe = sd.BandGatherPipeline(mk, rank, world, gather_fn,
                                     ops=sd.TorchStreamOps(stream_obj, comm, lambda h: ctx.wait_tail(h)))
    else:
        band_out = mk()
        gathered = ([mk() for _ in range(world)] if rank == 0 else None) if world > 1 else [mk()]
    torch.cuda.synchronize()

    # one step = one whole stack of the band, queued with sg_stack_u16_device_async on torch's
    # stream (every launch decided on the device, the counters read back into a pinned slot):
    # the host prepares the next step while the device runs this one.  Without a gather the
    # output is read after the timed region, so each step's work after its main kernel (redo list,
    # replay, counters) runs on the library's tail stream beside the next step
    # (SG_STACK_RESULT_AT_COLLECT)
    def step():
        if gathering and gather_mode == "overlap":
            pipe.step(lambda buf: ctx.stack_device_async(desc, base, fstride, nres * W, buf.data_ptr() - b * W * 2,
                                                         b, e, stream=stream))
        else:
            ctx.stack_device_async(desc, base, fstride, nres * W, band_out.data_ptr() - b * W * 2, b, e, stream=stream)
            if gathering:
                gather_fn(band_out, gathered)
        kms.append(ctx.stats().kernel_ms)       # the last folded call's (at most two calls behind)

    def reset_counters():
        rc, _, _ = ctx.collect()
        assert rc == 0, ctx.error()

    elapsed = timed(args.steps, args.warmup, step, D, after_warmup=reset_counters)
    rc, rej_steps, _ = ctx.collect()            # every timed step's counters, summed
    assert rc == 0, ctx.error()
    st = ctx.stats()
    kms.append(st.kernel_ms)
    kms = kms[args.warmup + 1:]
    kavg = sum(kms) / len(kms)
    per_rank_kms = D.all_floats(kavg)
    assert not (rej_steps % args.steps).any(), "the steps' rejection counters differ"
    rej_tot = rej_steps // args.steps           # one step's (every step stacks the same band)
    if world > 1:
        rej_tot = sd.sum_counters(rej_tot, D.dist, device=D.cdev)   # rejection counters, :1796-1817
    del frames
    torch.cuda.synchronize()
    torch.cuda.set_stream(prev_stream)
    torch.cuda.empty_cache()
    return {"elapsed": elapsed, "kavg": kavg, "per_rank_kms": per_rank_kms, "rej_tot": rej_tot, "st": st,
            "b": b, "e": e, "N": N, "H": H, "W": W, "Htot": Htot, "hband": hband, "nb": nb, "strong": strong,
            "median": median, "sig": sig, "gather": gather_mode if gathering else "none"}


def main_sigma(args):
    import numpy as np
    import torch
    import sirilgpu as sg
    D = Dist()
    world, rank = D.world, D.rank
    dev = torch.cuda.current_device()
    ctx = sg.Context([dev])
    strong = args.scaling == "strong" or world == 1
    gmode = args.strong_gather if (world > 1 or args.band_of > 1) else "none"
    f = sigma_form(args, ctx, D, strong, gmode)
    # at N > 1 in the (default) weak form, configs[3]'s strong form is timed after it and reported
    # beside it: the one 512-frame 4096-row sequence in N row bands, gathered to rank 0
    f_strong = sigma_form(args, ctx, D, True, args.strong_gather) if world > 1 and not strong else None
    N, H, W, b, e = f["N"], f["H"], f["W"], f["b"], f["e"]
    elapsed, kavg, st, median = f["elapsed"], f["kavg"], f["st"], f["median"]
    ms_step = elapsed / args.steps * 1e3
    frames_per_s = N * (1 if strong else world) / (elapsed / args.steps)
    algo_bytes = N * (e - b) * W * 2 + (e - b) * W * 2     # this rank's launch: its band's samples + output
    achieved = algo_bytes / (kavg * 1e-3) / 1e9
    if rank == 0:
        nb, hband, Htot, sig = f["nb"], f["hband"], f["Htot"], f["sig"]
        kind = "median stack" if median else f"{args.rejection} rejection stack"
        if world == 1 and nb > 1:
            workload = (f"A/B: band 0 ({e - b} rows) of the {kind} {N}x{H}x{W} u16 mono split into {nb} row bands "
                        f"(one rank's call of BASELINE configs[3] at {nb} GPUs), only its rows resident; "
                        f"value = frames/s of this band's work; gather stand-in: {f['gather']} "
                        f"(a {hband * W * 2}-byte device copy per step)")
            par = f"1 GPU, one of {nb} row bands"
        elif world == 1:
            workload = (f"{kind} {N}x{H}x{W} u16 mono (BASELINE configs[2] frames)" if median or args.rejection != "sigma"
                        else f"sigma-clip stack {N}x{H}x{W} u16 mono (BASELINE configs[2])")
            par = "1 GPU"
        elif strong:
            workload = (f"{kind} {N}x{H}x{W} u16 mono in {world} row bands of {hband} rows, output "
                        f"gathered to rank 0 (BASELINE configs[3], gather {f['gather']})")
            par = f"row-band x{world}, RCCL gather ({f['gather']})"
        else:
            workload = f"{kind} {N}x{H}x{W} u16 mono per GPU, one {N}x{Htot}x{W} sequence in {world} bands"
            par = f"row-band x{world} (weak)"
        res = {
            "metric": "frames/sec stacked (4096x4096 u16, sigma-clip) + achieved HBM GB/s",
            "value": round(frames_per_s, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong and world > 1 else args.scaling,   # at N = 1 both forms are one workload
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (include/sg_synth.h, generated in HBM)",
            "config": {"workload": workload, "frames": N, "height": H, "width": W,
                       "method": "median" if median else "mean", "rejection": "none" if median else args.rejection,
                       "sig": list(sig), "normalize": args.normalize, "parallelism": par},
            "roofline": roofline(achieved, algo_bytes, N, H, W, ("median" if median else args.rejection)
                                 if args.normalize == "none" else f"{'median' if median else args.rejection}_{args.normalize}",
                                 with_traffic=world == 1 and nb == 1),
            "kernel_ms": round(kavg, 3),
            "slow_pixels": int(st.slow_pixels),
            "redo_pixels": int(st.chain_pixels),
            "compact_pixels": int(st.compact_pixels),
            "rejected": [int(x) for x in np.asarray(f["rej_tot"]).reshape(-1)[:2]],
            **({"norm_load": ["reference", "fma", "integer"][max(0, min(2, int(st.norm_fma)))]}
               if args.normalize != "none" else {}),
        }
        if world > 1:
            res["per_rank_kernel_ms"] = [round(x, 3) for x in f["per_rank_kms"]]
            res["rows_per_rank"] = e - b
        if f_strong is not None:
            fs = f_strong
            res["configs3_strong"] = {
                "workload": f"{kind} {N}x{H}x{W} u16 mono (BASELINE configs[3]) in {world} row bands of "
                            f"{fs['hband']} rows, output bands gathered to rank 0 over RCCL ({fs['gather']})",
                "value": round(N / (fs["elapsed"] / args.steps), 2), "unit": "frames/s",
                "ms_per_step": round(fs["elapsed"] / args.steps * 1e3, 3), "scaling": "strong",
                "per_rank_kernel_ms": [round(x, 3) for x in fs["per_rank_kms"]],
                "rejected": [int(x) for x in np.asarray(fs["rej_tot"]).reshape(-1)[:2]]}
        if not args.no_cpu_baseline and world == 1 and nb == 1:
            res["cpu_baseline"] = cpu_baseline(args, N, W, median)
        print(json.dumps(res), flush=True)
    ctx.close()
    D.close()


def stack_roofline(achieved, algo_bytes, rej, N, C, H, W, world):
    """roofline of main_config's stack kernel; traffic = the PMC FETCH/WRITE bytes per launch
    of the whole image (profiles/traffic_{winsorized|mean}_<N>x<C>x<H>x<W>.json, 1 GPU)"""
    import sirilgpu as sg
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": "stack"}
    name = "winsorized" if rej == sg.WINSORIZED else "mean"
    path = os.path.join(ROOT, "profiles", f"traffic_{name}_{N}x{C}x{H}x{W}.json")
    t = load_traffic(path, r) if world == 1 else None
    if t is not None:
        r["traffic"] = int(t["traffic_bytes"])
        r["traffic_unit"] = "B/launch"
        r["traffic_over_algorithmic"] = round(t["traffic_bytes"] / algo_bytes, 4)
    return r


def main_config(args):
    """configs[1] (register-mean) and configs[4] (winsorized-rgb): one step = registration +
    stack; at N GPUs the registration is sharded over frames and the stack over row bands"""
    import numpy as np
    import torch
    import sirilgpu as sg
    import sirilgpu_dist as sd
    D = Dist()
    world, rank = D.world, D.rank
    dev = torch.cuda.current_device()
    ctx = sg.Context([dev])
    if args.workload == "register-mean":
        N, C, H, W, S, layer, rej, cfg = 128, 1, 2048, 2048, 2048, 0, sg.NO_REJEC, "BASELINE configs[1]"
    else:
        N, C, H, W, S, layer, rej, cfg = 256, 3, 4000, 6000, 2048, 1, sg.WINSORIZED, "BASELINE configs[4]"
    if args.selection:
        S = args.selection
        if not 2 <= S <= min(H, W):
            raise SystemExit(f"--selection {S} does not fit a {H}x{W} frame")
    seed, M = 0x5EED, 16
    y0, x0 = (H - S) // 2, (W - S) // 2
    ex, ey = synth_shifts_np(N, seed, M)
    # registration shard: the reference (frame 0) + this rank's frame block (without frame 0),
    # layer `layer`'s selection rows of every channel up to `layer` held compactly
    fb, fe = sd.frame_band(rank, world, N)
    mine = [f for f in range(fb, fe) if f != 0]
    nsel = 1 + len(mine)
    Cs = layer + 1
    selsrc = torch.empty(nsel * Cs * S * W, dtype=torch.int16, device="cuda")
    sbase = selsrc.data_ptr() - y0 * W * 2
    ctx.synth_fill(sbase, 1, Cs, H, W, y0, y0 + S, seed, M, frame_stride=Cs * S * W, plane_stride=S * W)
    if mine:
        ctx.synth_fill(sbase + Cs * S * W * 2, len(mine), Cs, H, W, y0, y0 + S, seed, M, frame_stride=Cs * S * W,
                       plane_stride=S * W, first_frame=mine[0])
    # stack shard: row band of every frame (band + shift halo), all channels
    b, e = sd.row_band(rank, world, H)
    lo, hi = max(0, b - int(ey.max())), min(H - 1, e - 1 - int(ey.min()))
    nres = hi - lo + 1
    fstride = C * nres * W
    frames = torch.empty(N * fstride, dtype=torch.int16, device="cuda")
    fbase = frames.data_ptr() - lo * W * 2
    ctx.synth_fill(fbase, N, C, H, W, lo, hi + 1, seed, M, frame_stride=fstride, plane_stride=nres * W)
    hband = -(-H // world)
    # the library writes rows [b, e) of every channel of a [C][H][W] image; the channels' bands
    # are packed into one send buffer for the gather
    out_img = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    band_out = torch.zeros(C * hband * W, dtype=torch.int16, device="cuda")
    gathered = None
    if world > 1 and rank == 0:
        gathered = [torch.empty(C * hband * W, dtype=torch.int16, device="cuda") for _ in range(world)]
    torch.cuda.synchronize()
    stage = np.zeros(3)
    kms = []
    reg_spans = []
    out = {}

    # seq_read_frame_part of layer `layer`: the S x S windows read in place by the registration's
    # first pass (sg_register_dft_u16_device_pitched; round 5 extracted them with a 2 x 2 GB copy
    # first, the "selection" stage, 1.47 ms of configs[4]'s step)
    sel_base = selsrc.data_ptr() + 2 * (layer * S * W + x0)

    def step():
        t0 = time.perf_counter()
        t1 = time.perf_counter()
        lx, ly, lq = ctx.register_dft_device(sel_base, nsel, S, raw_quality=world > 1, frame_pitch=Cs * S * W,
                                             row_pitch=W)
        reg_spans.append(ctx.stats().reg_ms)
        if world > 1:
            rows = np.zeros((3, N))
            for k, f in enumerate(mine):
                rows[:, f] = lx[k + 1], ly[k + 1], lq[k + 1]
            if rank == 0:
                rows[2, 0] = lq[0]
            t = torch.as_tensor(rows, device=D.cdev)
            D.dist.all_reduce(t)                          # disjoint frame blocks: the sum is the gather
            rows = t.cpu().numpy()
            sx, sy = rows[0].astype(np.int32), rows[1].astype(np.int32)
            q = sd.normalize_quality(rows[2], N, 0, None)
        else:
            sx, sy, q = lx, ly, lq
        t2 = time.perf_counter()
        if world == 1:
            # queued (sg_stack_u16_device_async, SG_STACK_RESULT_AT_COLLECT): the stack's work after its
            # main kernel (the replay of early-break / redo pixels) runs on the library's tail stream
            # beside the next step's registration, which follows the main kernel on the call's stream;
            # the counters of every step come back with one collect after the timed region (the
            # configs[2] step's scheme)
            desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=rej, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                      max_thread=8, max_number_of_rows=H, resident_rows=(lo, hi + 1),
                                      flags=sg.RESULT_AT_COLLECT)
            ctx.stack_device_async(desc, fbase, fstride, nres * W, out_img.data_ptr(), b, e,
                                   stream=side.cuda_stream if side is not None else None)
            kms.append(ctx.stats().kernel_ms)       # the last folded call's
            stage_keep.append(keep)
            t3 = time.perf_counter()
            stage[:] += (t1 - t0, t2 - t1, t3 - t2)
            out["sx"], out["sy"] = sx, sy
            return
        desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=rej, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                  max_thread=8, max_number_of_rows=H, resident_rows=(lo, hi + 1))
        rj, _ = ctx.stack_device(desc, fbase, fstride, nres * W, out_img.data_ptr(), b, e)
        kms.append(ctx.stats().kernel_ms)
        if world > 1:
            band_out.view(C, hband, W)[:, :e - b].copy_(out_img.view(C, H, W)[:, b:e])
            D.gather_to_root(band_out, gathered)
            D.sum_counters(rj)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        stage[:] += (t1 - t0, t2 - t1, t3 - t2)
        out["sx"], out["sy"] = sx, sy

    stage_keep = []         # the queued calls' descriptors (their arrays) stay alive until collected
    # the stack's own stream: step k's stack kernel (it needs step k's shifts, so it is queued once the
    # registration has returned) runs beside step k+1's registration passes, which do not read it
    side = torch.cuda.Stream() if world == 1 and args.stack_stream == "side" else None
    for _ in range(args.warmup):
        step()
    if world == 1:
        torch.cuda.synchronize()
        rc, _, _ = ctx.collect()
        assert rc == 0, ctx.error()
        stage_keep.clear()
    stage[:] = 0
    kms.clear()
    reg_spans.clear()
    elapsed = timed(args.steps, 0, step, D)
    stage /= args.steps
    if world == 1:      # every timed step's counters; the statistics of the last call
        rc, rej_all, _ = ctx.collect()
        assert rc == 0, ctx.error()
        stage_keep.clear()
        kms.append(ctx.stats().kernel_ms)
        kms = kms[1:]   # the first entry described a warm-up call
    reg_ok = bool(np.array_equal(out["sx"], ex) and np.array_equal(out["sy"], ey))
    kavg = sum(kms) / len(kms)
    stack_bytes = N * C * (e - b) * W * 2 + C * (e - b) * W * 2
    achieved = stack_bytes / (kavg * 1e-3) / 1e9
    # registration roofline: algorithmic bytes of the half-spectrum fp32 pass structure (DESIGN.md
    # section 2, Registration): per pair of frames the two u16 selections (4 S^2), the pair plane
    # written and read back by the column pass (8 + 8 S^2), the reference's half spectrum (4 S^2),
    # the column pass's output read by the inverse rows (8 + 8 S^2): 40 S^2 per pair = 20 S^2 per
    # frame, plus the quality estimate's read of the selection (2 S^2; at S = 2048 the forward rows
    # subsample the selections they read (SG_REG_QFOLD, default on), so the estimate adds only its
    # subsampled frames written and read back, 2 x 2 (S / 3)^2 = 4/9 S^2); the measured PMC bytes
    # are the traffic
    qfold = S == 2048 and int(os.environ.get("SG_REG_QFOLD", "12")) >= 3
    reg_algo = int(nsel * S * S * (20 + 4 / 9 if qfold else 22))
    reg_ms = sum(reg_spans) / len(reg_spans) if reg_spans else stage[1] * 1e3
    tpath = os.path.join(ROOT, "profiles", f"traffic_register_{N}x{S}.json")
    reg_tinfo = {}
    reg_traffic = load_traffic(tpath, reg_tinfo) if world == 1 else None
    if rank == 0:
        res = {
            "metric": "frames/sec stacked (registration + stack) + achieved HBM GB/s",
            "value": round(N / (elapsed / args.steps), 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u16",
            "data": "synthetic (include/sg_synth.h, generated in HBM)",
            "config": {"workload": f"{args.workload} {N}x{C}x{H}x{W} ({cfg})" +
                       (f", {S}^2 selection" if args.selection else ""), "frames": N, "layers": C,
                       "height": H, "width": W, "selection": S, "register_layer": layer,
                       "rejection": "none" if rej == sg.NO_REJEC else "winsorized",
                       "parallelism": "1 GPU" if world == 1 else
                       f"registration frame-sharded x{world} + stack row-band x{world}, RCCL gather"},
            "stage_ms": {"selection": round(stage[0] * 1e3, 3), "register": round(stage[1] * 1e3, 3),
                         "stack_mode": ("queued on a second stream: host time to queue the stack; its main kernel "
                                        "runs beside the next step's registration" if side is not None else
                                        "queued on the registration's stream: host time to queue the stack; its tail "
                                        "runs beside the next step's registration") if world == 1 else "synchronous",
                         "register_device": round(reg_ms, 3), "stack": round(stage[2] * 1e3, 3),
                         "stack_kernel": round(kavg, 3)},
            "register_shifts_exact": reg_ok,
        }
        # the roofline object describes the step's dominant stage (configs[1]: the registration
        # passes; configs[4]: the Winsorized stack kernel), the other stage's as a second field
        reg_ach = reg_algo / (reg_ms * 1e-3) / 1e9
        rr = {"bound": "hbm", "kernel": "registration passes (device span: rows, columns + cross power, inverse "
                                        "rows + arg-max, quality estimate)",
              "achieved": round(reg_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(reg_ach / HBM_PEAK_GBS, 4), "algorithmic_bytes": int(reg_algo),
              "algorithmic_model": "20 4/9 S^2 per frame (DESIGN.md: 20 S^2 FFT passes + 4/9 S^2 quality, subsample "
                                   "folded into the forward rows)" if qfold else
                                   "22 S^2 per frame (DESIGN.md: 20 S^2 FFT passes + 2 S^2 quality)",
              "traffic": None}
        # SURVEY 8(d)'s algorithmic MINIMUM: each u16 selection read once (2 S^2 per frame); the
        # passes' planes cannot stay on chip at S = 2048 (32 MiB per c64 plane), so this is a floor
        # no pass structure reaches, reported beside the pass model
        reg_min = nsel * S * S * 2
        rr["min_model"] = {"algorithmic_bytes": int(reg_min), "model": "2 S^2 per frame (SURVEY 8(d) minimum)",
                           "achieved": round(reg_min / (reg_ms * 1e-3) / 1e9, 1),
                           "frac": round(reg_min / (reg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if reg_traffic is not None:
            # PMC FETCH/WRITE bytes of the registration kernels per step (scripts/pmc_traffic.py)
            tb = reg_traffic["traffic_bytes_per_step"]
            rr["traffic"] = int(tb)
            rr["traffic_unit"] = "B/step"
            rr["traffic_over_algorithmic"] = round(tb / reg_algo, 4)
            rr["traffic_GBps"] = round(tb / (reg_ms * 1e-3) / 1e9, 1)
        rr.update(reg_tinfo)
        sr = stack_roofline(achieved, stack_bytes, rej, N, C, H, W, world)
        if reg_ms >= kavg:
            res["roofline"], res["stack_roofline"] = rr, sr
        else:
            res["roofline"], res["register_roofline"] = sr, rr
        if S & (S - 1):
            res["cpu_baseline_note"] = "none: the oracle's radix-2 DFT takes power-of-two sides only"
        if not args.no_cpu_baseline and world == 1 and (S & (S - 1)) == 0:
            res["cpu_baseline"] = cpu_baseline_config(args, args.workload, N, C, H, W, S, layer)
        print(json.dumps(res), flush=True)
    ctx.close()
    D.close()


def main_sum(args):
    """configs[0]: stack_summing of 16 x 1024^2 u16 mono FITS frames, end to end from the files
    through the library's FITS region reader (sg_stack_u16, the drop-in host-pull path)"""
    import tempfile
    import numpy as np
    import torch
    import sirilgpu as sg
    from seq_files import write_fits
    D = Dist()
    N, C, H, W, M = 16, 1, 1024, 1024, 16
    ctx = sg.Context([0])
    # frames from the library's generator (include/sg_synth.h) through HBM to the host; the
    # oracle runs only in the CPU-baseline leg below (timing and the check of the result)
    d_gen = torch.empty(N * C * H * W, dtype=torch.int16, device="cuda")
    ctx.synth_fill(d_gen.data_ptr(), N, C, H, W, 0, H, 0xF175, M)
    frames = d_gen.cpu().numpy().view(np.uint16).reshape(N, C, H, W)
    del d_gen
    sx, sy = synth_shifts_np(N, 0xF175, M)
    with tempfile.TemporaryDirectory() as tmp:
        paths = []
        for i in range(N):
            p = os.path.join(tmp, f"light_{i + 1:05d}.fit")
            write_fits(p, frames[i])
            paths.append(p)
        desc, keep = sg.make_desc(sg.SUM, N, W, H, C, shiftx=sx, shifty=sy)
        with sg.Seq.open_fits(paths) as seq:
            res_out = {}

            def step():
                rc, out, _, maxim = ctx.stack_seq(desc, seq)
                assert rc == 0, ctx.error()
                res_out["out"] = out

            elapsed = timed(args.steps, args.warmup, step, D)
    res = {
        "metric": "frames/sec stacked (stack_summing, end to end from FITS files)",
        "value": round(N / (elapsed / args.steps), 2), "unit": "frames/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u16",
        "data": "synthetic frames written as FITS files (BITPIX 16, BZERO 32768) in a temporary directory",
        "config": {"workload": f"stack_summing {N}x{H}x{W} u16 mono FITS (BASELINE configs[0]), host-pull from "
                               f"files (reads + decode + PCIe + kernels)", "parallelism": "1 GPU"},
    }
    if not args.no_cpu_baseline:
        import oracle_lib as orc
        rc, ref, _ = orc.stack_sum(frames, sx, sy)
        res["matches_oracle"] = bool(np.array_equal(res_out["out"], ref))
        _omp_threads(1)
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            orc.stack_sum(frames, sx, sy)
        dt = (time.perf_counter() - t0) / reps
        res["cpu_baseline"] = {"value": round(N / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                               "cpu_model": cpu_model(),
                               "sample": f"oracle stack_summing (single thread, as the reference's :196-355), the "
                                         f"same {N} frames RAM-resident ({reps} runs)"}
    print(json.dumps(res), flush=True)
    ctx.close()
    D.close()


def main_register_file(args):
    """configs[1] end to end from a file: a 128-frame 2048^2 u16 SER written once, then per step
    sg_seq_load_device (file bytes through pinned staging, PCIe, device decode into Siril's
    bottom-up layout) + register_shift_dft on the full-frame selection + the mean stack with the
    shifts - the drop-in host path's figure against the PCIe roofline (never the headline)"""
    import tempfile
    import numpy as np
    import torch
    import sirilgpu as sg
    from seq_files import write_ser
    D = Dist()
    N, C, H, W, seed, M = 128, 1, 2048, 2048, 0x5EED, 16
    ex, ey = synth_shifts_np(N, seed, M)
    ctx = sg.Context([torch.cuda.current_device()])
    d_frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
    # the library's own generator (include/sg_synth.h), copied to the host for the file
    ctx.synth_fill(d_frames.data_ptr(), N, C, H, W, 0, H, seed, M)
    frames = d_frames.cpu().numpy().view(np.uint16).reshape(N, C, H, W)
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    stage = np.zeros(3)
    got = {}
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "light.ser")
        write_ser(path, frames, depth=16)
        del frames
        with sg.Seq.open_ser(path) as seq:
            def step():
                t0 = time.perf_counter()
                ctx.load_seq_device(seq, d_frames.data_ptr())
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                sx, sy, q = ctx.register_dft_device(d_frames.data_ptr(), N, W)
                t2 = time.perf_counter()
                desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, shiftx=sx, shifty=sy, max_thread=8,
                                          max_number_of_rows=H)
                ctx.stack_device(desc, d_frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
                torch.cuda.synchronize()
                t3 = time.perf_counter()
                stage[:] += (t1 - t0, t2 - t1, t3 - t2)
                got["sx"], got["sy"] = sx, sy

            for _ in range(args.warmup):
                step()
            stage[:] = 0
            elapsed = timed(args.steps, 0, step, D)
    stage /= args.steps
    file_bytes = N * H * W * 2
    res = {
        "metric": "frames/sec registered + mean-stacked, end to end from a SER file",
        "value": round(N / (elapsed / args.steps), 2), "unit": "frames/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u16",
        "data": "synthetic frames (include/sg_synth.h generator) written once as a 16-bit mono SER in a temporary "
                "directory (page-cache resident after the write)",
        "config": {"workload": f"register-mean {N}x{H}x{W} (BASELINE configs[1]) from a SER file: "
                               "sg_seq_load_device + register_shift_dft (full-frame selection) + mean",
                   "parallelism": "1 GPU"},
        "stage_ms": {"load": round(stage[0] * 1e3, 3), "register": round(stage[1] * 1e3, 3),
                     "stack": round(stage[2] * 1e3, 3)},
        "load_GBps": round(file_bytes / stage[0] / 1e9, 1),
        "register_shifts_exact": bool(np.array_equal(got["sx"], ex) and np.array_equal(got["sy"], ey)),
    }
    print(json.dumps(res), flush=True)
    ctx.close()
    D.close()


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    if os.environ.get("SG_BENCH_LAUNCH_PROBE") == "1":     # tests: report the rank layout, touch no GPU
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": int(os.environ.get("WORLD_SIZE", "1")),
                          "gpus": args.gpus}), flush=True)
        return
    if args.workload in ("sigma", "median"):
        return main_sigma(args)
    if args.workload == "sum-fits":
        return main_sum(args)
    if args.workload == "register-mean-file":
        return main_register_file(args)
    return main_config(args)


if __name__ == "__main__":
    main()
