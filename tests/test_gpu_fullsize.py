"""Every BASELINE.json configuration at its full size, on the GPU, checked against the C
oracle and against golden registration results (tests/golden/make_golden_fullsize.py).

  configs[0]  stack_summing of 16 x 1024 x 1024 u16 mono FITS files, from the files
  configs[1]  128 x 2048 x 2048 u16 mono SER file: device load, full-frame DFT registration,
              NO_REJEC mean stack with the found shifts (device and host-pull paths)
  configs[2]  SIGMA (4, 3) stack of 512 x 4096 x 4096, the WHOLE image against the oracle; the
              same frames' whole stack_median and PERCENTILE images (histogram rank path)
  configs[3]  the same stack as 8 row bands (the multi-GPU partition, band-only residency
              windows) equal to the one-call image
  configs[4]  256 x 3 x 4000 x 6000: DFT registration of layer 1's centred 2048 selection,
              WINSORIZED (4, 3) stack of all three channels with those shifts: the whole image
              against the independent sorted-kernel path, sampled row bands of every channel
              against the oracle

Frames are the synthetic sequence of include/sg_synth.h (generated in HBM by the library,
and by the oracle for the golden files).  At these frame counts no first sigma pass breaks
early, so the oracle's OpenMP thread order (which only matters for stale rejected[]) cannot
change a pixel, and a row band of the oracle's image equals the oracle run on that band plus
its 16-row shift halo (the y shift is a translation with zero fill,
src/stacking/stacking.c:1550-1577).
"""
import os
import sys

import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg
import sirilgpu_dist as sd
from seq_files import write_fits, write_ser

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def normalize_quality(raw, ref_image=0, included=None):
    """normalizeQualityData (src/registration/registration.c:163-176) with q_min / q_max as
    register_shift_dft forms them (:270-324: seeded by the reference, then frames in index
    order, siril.h's min() macro)"""
    n = len(raw)
    inc = np.ones(n, bool) if included is None else np.asarray(included, bool)
    q_min = q_max = raw[ref_image]
    for f in range(n):
        if f == ref_image or not inc[f]:
            continue
        q = raw[f]
        if q > q_max:
            q_max = q
        q_min = q_min if q_min < q else q
    out = raw.copy()
    for f in range(n):
        if inc[f]:
            out[f] = (raw[f] - q_min) / (q_max - q_min)
    return out


def _free():
    import torch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_cfg0_fits_summing_from_files(tmp_path, gpu_ctx):
    """configs[0]: stack_summing (src/stacking/stacking.c:196-355) of 16 x 1024^2 FITS files with
    registration shifts, fed by the library's FITS region reader (host-pull) and by the device
    decode path; the 65535/max scaling applies (16 frames of ~1000 ADU)"""
    import torch
    N, C, H, W, M = 16, 1, 1024, 1024, 16
    frames = orc.synth(N, C, H, W, seed=0xF175, maxshift=M)
    sx, sy = orc.synth_shifts(N, seed=0xF175, maxshift=M)
    paths = []
    for i in range(N):
        p = str(tmp_path / f"light_{i + 1:05d}.fit")
        write_fits(p, frames[i])
        paths.append(p)
    rc, ref, mref = orc.stack_sum(frames, sx, sy)
    assert rc == 0 and mref > 65535
    desc, keep = sg.make_desc(sg.SUM, N, W, H, C, shiftx=sx, shifty=sy)
    with sg.Seq.open_fits(paths) as seq:
        rc, out, _, maxim = gpu_ctx.stack_seq(desc, seq)
        assert rc == 0, gpu_ctx.error()
        assert maxim == mref
        assert np.array_equal(out, ref)
        d = torch.zeros(N * C * H * W, dtype=torch.int16, device="cuda")
        o = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.load_seq_device(seq, d.data_ptr())
        _, m2 = gpu_ctx.stack_device(desc, d.data_ptr(), C * H * W, H * W, o.data_ptr(), 0, H)
        assert m2 == mref
        assert np.array_equal(o.cpu().numpy().view(np.uint16).reshape(C, H, W), ref)


def test_cfg1_ser_register_mean(tmp_path, gpu_ctx):
    """configs[1]: a 128 x 2048^2 SER file written the way ser_write_frame_from_fit does,
    decoded into HBM, registered on the full frame, mean-stacked with the found shifts"""
    import torch
    g = np.load(os.path.join(GOLDEN, "register_cfg1.npz"))
    N, C, H, W, layer, S, y0, x0, seed, M = (int(v) for v in g["geometry"])
    fr = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
    gpu_ctx.synth_fill(fr.data_ptr(), N, 1, H, W, 0, H, seed, M)
    frames = fr.cpu().numpy().view(np.uint16).reshape(N, 1, H, W)
    path = str(tmp_path / "cfg1.ser")
    write_ser(path, frames, depth=16)
    loaded = torch.zeros(N * H * W, dtype=torch.int16, device="cuda")
    with sg.Seq.open_ser(path) as seq:
        assert seq.shape == (N, 1, H, W)
        torch.cuda.synchronize()
        gpu_ctx.load_seq_device(seq, loaded.data_ptr())
        assert torch.equal(loaded, fr), "SER decode differs from the generated frames"
        # registration (full-frame selection: the decoded frames themselves)
        sx, sy, q = gpu_ctx.register_dft_device(loaded.data_ptr(), N, S)
        assert np.array_equal(sx, g["shiftx"]) and np.array_equal(sy, g["shifty"]), "shifts differ from golden"
        _, _, qraw = gpu_ctx.register_dft_device(loaded.data_ptr(), N, S, raw_quality=True)
        assert np.array_equal(qraw, g["quality_raw"]), "raw quality differs from golden"
        assert np.array_equal(q, normalize_quality(g["quality_raw"])), "normalised quality differs"
        # NO_REJEC mean with the found shifts, device path and host-pull path (the SER region reader)
        rc, ref, _ = orc.stack_rejection(frames, sg.NO_REJEC, shiftx=sx, shifty=sy, max_thread=16)
        assert rc == 0
        desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.NO_REJEC, shiftx=sx, shifty=sy,
                                  max_thread=16, max_number_of_rows=H)
        o = torch.zeros(H * W, dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.stack_device(desc, loaded.data_ptr(), H * W, H * W, o.data_ptr(), 0, H)
        assert np.array_equal(o.cpu().numpy().view(np.uint16).reshape(1, H, W), ref)
        rc, out, _, _ = gpu_ctx.stack_seq(desc, seq)
        assert rc == 0, gpu_ctx.error()
        assert np.array_equal(out, ref)
    del fr, loaded, o
    _free()


def _sigma_cfg2(gpu_ctx):
    import torch
    import bench
    N, H, W, M = 512, 4096, 4096, 16
    frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
    gpu_ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, M)
    sx, sy = bench.synth_shifts_np(N, 0x5151, M)
    return frames, sx, sy, (N, H, W, M)


def test_cfg2_sigma_whole_image_and_cfg3_bands(gpu_ctx):
    """configs[2] (the headline workload): the whole 512 x 4096^2 SIGMA (4, 3) image and the
    rejection counters against the oracle; configs[3]'s partition (8 row bands, each call with
    only its band's rows + shift halo declared resident) equal to the one-call image"""
    import torch
    frames, sx, sy, (N, H, W, M) = _sigma_cfg2(gpu_ctx)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              max_thread=16, max_number_of_rows=H)
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rej, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    img = out.cpu().numpy().view(np.uint16).reshape(H, W)
    # configs[3]: 8 bands, each with a resident window of its rows + halo (no copies: the
    # window is declared on the whole buffer, so any read outside it is refused, not served)
    G = 8
    out8 = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rej8 = np.zeros((3, 2), np.uint64)
    for r in range(G):
        b, e = sd.row_band(r, G, H)
        lo, hi = max(0, b - int(sy.max())), min(H - 1, e - 1 - int(sy.min()))
        d8, k8 = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              max_thread=16, max_number_of_rows=H, resident_rows=(lo, hi + 1))
        rj, _ = gpu_ctx.stack_device(d8, frames.data_ptr(), H * W, H * W, out8.data_ptr(), b, e)
        rej8 += rj
    assert torch.equal(out8, out), "8-band stack differs from the one-call stack"
    assert np.array_equal(rej8, rej)
    host = frames.cpu().numpy().view(np.uint16).reshape(N, 1, H, W)
    del frames, out, out8
    _free()
    rc, ref, rej_ref = orc.stack_rejection(host, sg.SIGMA, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           max_thread=16, max_number_of_rows=H)
    assert rc == 0
    bad = np.argwhere(img != ref[0])
    assert bad.size == 0, f"{len(bad)} pixels differ from the oracle, first {bad[:3].tolist()}"
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


def test_cfg2_median_and_percentile_whole_image(gpu_ctx):
    """configs[2]'s frames through the histogram rank path of stack_median
    (src/stacking/stacking.c:746-767) and PERCENTILE (0.2, 0.1) rejection (:1660-1673), the whole
    512 x 4096^2 image (and the counters) against the oracle"""
    import torch
    frames, sx, sy, (N, H, W, M) = _sigma_cfg2(gpu_ctx)
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    dmed, km = sg.make_desc(sg.MEDIAN, N, W, H, 1, max_thread=16, max_number_of_rows=H)
    torch.cuda.synchronize()
    gpu_ctx.stack_device(dmed, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    assert gpu_ctx.stats().path == 1
    med = out.cpu().numpy().view(np.uint16).reshape(H, W).copy()
    dpct, kp = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.PERCENTILE, sig=(0.2, 0.1), shiftx=sx, shifty=sy,
                            max_thread=16, max_number_of_rows=H)
    rej, _ = gpu_ctx.stack_device(dpct, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    assert gpu_ctx.stats().path == 1
    pct = out.cpu().numpy().view(np.uint16).reshape(H, W)
    host = frames.cpu().numpy().view(np.uint16).reshape(N, 1, H, W)
    del frames, out
    _free()
    rc, ref = orc.stack_median(host, max_thread=16, max_number_of_rows=H)
    assert rc == 0
    bad = np.argwhere(med != ref[0])
    assert bad.size == 0, f"median: {len(bad)} pixels differ from the oracle, first {bad[:3].tolist()}"
    del ref
    rc, ref, rej_ref = orc.stack_rejection(host, sg.PERCENTILE, sig=(0.2, 0.1), shiftx=sx, shifty=sy,
                                           max_thread=16, max_number_of_rows=H)
    assert rc == 0
    bad = np.argwhere(pct != ref[0])
    assert bad.size == 0, f"percentile: {len(bad)} pixels differ from the oracle, first {bad[:3].tolist()}"
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


def test_cfg4_rgb_register_and_winsorized(gpu_ctx):
    """configs[4] on one GPU: 256 x 3 x 4000 x 6000 frames in HBM, DFT registration of layer 1's
    centred 2048 selection (golden shifts and qualities), WINSORIZED (4, 3) stack of all three
    channels with the found shifts, the whole image against the sort-based kernel path and 3 row
    bands of every channel against the oracle"""
    import torch
    g = np.load(os.path.join(GOLDEN, "register_cfg4.npz"))
    N, C, H, W, layer, S, y0, x0, seed, M = (int(v) for v in g["geometry"])
    frames = torch.empty(N * C * H * W, dtype=torch.int16, device="cuda")
    gpu_ctx.synth_fill(frames.data_ptr(), N, C, H, W, 0, H, seed, M)
    fv = frames.view(N, C, H, W)
    sel = fv[:, layer, y0:y0 + S, x0:x0 + S].contiguous()     # seq_read_frame_part of layer 1
    torch.cuda.synchronize()
    sx, sy, q = gpu_ctx.register_dft_device(sel.data_ptr(), N, S)
    assert np.array_equal(sx, g["shiftx"]) and np.array_equal(sy, g["shifty"]), "shifts differ from golden"
    _, _, qraw = gpu_ctx.register_dft_device(sel.data_ptr(), N, S, raw_quality=True)
    assert np.array_equal(qraw, g["quality_raw"])
    assert np.array_equal(q, normalize_quality(g["quality_raw"]))
    del sel
    # 3 oracle bands of 64 rows per channel (the top and bottom ones with the zero fill of rows
    # shifted out of the frame, the middle one; two more per channel in the next test), run on
    # the host in a thread while the GPU stacks the image on both kernel paths
    starts = [0, H // 2 - 32, H - 64]
    jobs = []
    for c in range(C):
        for b in starts:
            lo, hi = max(0, b - M), min(H, b + 64 + M)
            jobs.append((c, b, lo, fv[:, c, lo:hi, :].cpu().numpy().view(np.uint16)[:, None]))

    def oracle_bands():
        res = []
        for c, b, lo, band in jobs:
            rc, ref, _ = orc.stack_rejection(band, sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                             max_thread=16, max_number_of_rows=16 * 24)
            res.append((c, b, lo, rc, ref[0, b - lo:b + 64 - lo].copy()))
        return res

    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(1)
    fut = pool.submit(oracle_bands)
    out = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              max_thread=16, max_number_of_rows=H)
    rej, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), C * H * W, H * W, out.data_ptr(), 0, H)
    assert gpu_ctx.stats().path == 1
    # the WHOLE image (all 3 channels) against the independent sort-based kernel path
    # (k_stack_sorted + replay + literal, each checked against the oracle at small sizes)
    d_s, k_s = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                            max_thread=16, max_number_of_rows=H, kernel_path=sg.PATH_SORTED)
    out_s = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rej_s, _ = gpu_ctx.stack_device(d_s, frames.data_ptr(), C * H * W, H * W, out_s.data_ptr(), 0, H)
    assert gpu_ctx.stats().path == 0
    nbad = int((out_s != out).sum())
    assert nbad == 0, f"{nbad} pixels differ between the histogram and the sorted kernel paths"
    assert np.array_equal(rej_s, rej), (rej_s, rej)
    del out_s
    img = out.cpu().numpy().view(np.uint16).reshape(C, H, W)
    for c, b, lo, rc, want in fut.result():
        assert rc == 0
        got = img[c, b:b + 64]
        bad = np.argwhere(got != want)
        assert bad.size == 0, f"channel {c} rows {b}..{b + 64}: {len(bad)} pixels differ, first {bad[:3].tolist()}"
    pool.shutdown()
    del frames, out, fv
    _free()


def test_cfg4_winsorized_more_oracle_bands(gpu_ctx):
    """configs[4]'s WINSORIZED image (golden registration shifts) at two more 64-row bands per
    channel, at 1/4 and 3/4 of the height, against the oracle: with the previous test 5 bands per
    channel, 8 % of the image (the oracle's CPU time bounds the coverage per test)"""
    import torch
    g = np.load(os.path.join(GOLDEN, "register_cfg4.npz"))
    N, C, H, W, layer, S, y0, x0, seed, M = (int(v) for v in g["geometry"])
    sx, sy = g["shiftx"].astype(np.int32), g["shifty"].astype(np.int32)
    frames = torch.empty(N * C * H * W, dtype=torch.int16, device="cuda")
    gpu_ctx.synth_fill(frames.data_ptr(), N, C, H, W, 0, H, seed, M)
    out = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              max_thread=16, max_number_of_rows=H)
    gpu_ctx.stack_device(desc, frames.data_ptr(), C * H * W, H * W, out.data_ptr(), 0, H)
    assert gpu_ctx.stats().path == 1
    img = out.cpu().numpy().view(np.uint16).reshape(C, H, W)
    fv = frames.view(N, C, H, W)
    for c in range(C):
        for b in (H // 4 - 32, 3 * H // 4 - 32):
            lo, hi = max(0, b - M), min(H, b + 64 + M)
            band = fv[:, c, lo:hi, :].cpu().numpy().view(np.uint16)[:, None]
            rc, ref, _ = orc.stack_rejection(band, sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                             max_thread=16, max_number_of_rows=16 * 24)
            assert rc == 0
            bad = np.argwhere(img[c, b:b + 64] != ref[0, b - lo:b + 64 - lo])
            assert bad.size == 0, f"channel {c} rows {b}..{b + 64}: {len(bad)} pixels differ, first {bad[:3].tolist()}"
    del frames, out, fv
    _free()


def _oracle_band_jobs(fv, starts, rows, M, C=None):
    """host copies of the frame rows each 64-row band reads (band + M-row shift halo)"""
    jobs = []
    H = fv.shape[-2]
    for b in starts:
        lo, hi = max(0, b - M), min(H, b + rows + M)
        src = fv[:, lo:hi, :] if C is None else fv[:, C, lo:hi, :]
        jobs.append((b, lo, src.cpu().numpy().view(np.uint16)[:, None]))
    return jobs


@pytest.mark.parametrize("rejection", ["linearfit", "sigmedian"])
def test_cfg2_fast_kernels_oracle_bands(gpu_ctx, rejection):
    """configs[2]'s 512 x 4096^2 frames through the round-5 fast kernels, LINEARFIT (4, 3) on
    k_stack_linfit (stacking.c:1750-1784) and SIGMEDIAN (4, 3) on k_stack_hist<3> (:1696-1709), at
    full size.  The whole image is stacked in one call; 64 band calls of 64 rows repeat it (same
    image) and report each band's redo pixels (decisions inside the recurrence-error bound /
    rounding band, re-done by the sorted kernel's exact replay).  8 bands go to the oracle, run on
    host threads while the GPU works: the top and bottom bands (rows shifted out of the frames,
    zero fill) and the 6 bands with the MOST redo pixels, so the bound's edge is where the oracle
    looks; each band's image rows and its rejection counters (the oracle's per-row counts) must be
    equal, and for LINEARFIT the checked bands must hold redo pixels"""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    rj = {"linearfit": sg.LINEARFIT, "sigmedian": sg.SIGMEDIAN}[rejection]
    frames, sx, sy, (N, H, W, M) = _sigma_cfg2(gpu_ctx)
    fv = frames.view(N, H, W)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rj, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              max_thread=16, max_number_of_rows=H)
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    outb = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rej_all, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    st = gpu_ctx.stats()
    assert st.path == 1, "not on the fast kernel"
    redo_all = int(st.chain_pixels)
    R = 64
    band_rej, band_redo = {}, {}
    for b in range(0, H, R):
        r, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, outb.data_ptr(), b, b + R)
        band_rej[b] = r.copy()
        band_redo[b] = int(gpu_ctx.stats().chain_pixels)
    assert torch.equal(outb, out), "64 band calls differ from the one-call image"
    assert np.array_equal(sum(band_rej.values()), rej_all)
    assert sum(band_redo.values()) == redo_all, (sum(band_redo.values()), redo_all)
    inner = sorted((b for b in band_redo if 0 < b < H - R), key=lambda b: (-band_redo[b], b))
    starts = [0, H - R] + inner[:6]
    jobs = _oracle_band_jobs(fv, starts, R, M)

    def oracle_bands():
        res = []
        for b, lo, band in jobs:
            rc, ref, _, rows = orc.stack_rejection(band, rj, sig=(4.0, 3.0), shiftx=sx, shifty=sy, max_thread=16,
                                                   max_number_of_rows=16 * 24, row_counters=True)
            res.append((b, rc, ref[0, b - lo:b + R - lo].copy(), rows[0, b - lo:b + R - lo].sum(axis=0)))
        return res

    pool = ThreadPoolExecutor(1)
    fut = pool.submit(oracle_bands)
    img = out.cpu().numpy().view(np.uint16).reshape(H, W)
    checked_redo = sum(band_redo[b] for b in starts)
    for b, rc, want, rows in fut.result():
        assert rc == 0
        bad = np.argwhere(img[b:b + R] != want)
        assert bad.size == 0, f"{rejection} rows {b}..{b + R}: {len(bad)} pixels differ, first {bad[:3].tolist()}"
        assert np.array_equal(band_rej[b][0], rows), (b, band_rej[b][0], rows)
    pool.shutdown()
    print(f"{rejection}: redo pixels {redo_all} in the image, {checked_redo} in the 8 oracle bands "
          f"{[(b, band_redo[b]) for b in starts]}")
    if rj == sg.LINEARFIT:
        assert checked_redo > 0, "no redo pixel in the oracle bands: the bound's edge is not exercised"
    del frames, out, outb, fv
    _free()


@pytest.mark.parametrize("part", [0, 1])
def test_cfg4_winsorized_oracle_bands_spread(gpu_ctx, part):
    """configs[4]'s WINSORIZED image at 3 more 64-row bands per channel and part (6 over both
    parts, spread between the 5 of the two tests above), against the oracle run on a host thread
    while the GPU stacks: with them 11 bands per channel, 18 % of the image"""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    g = np.load(os.path.join(GOLDEN, "register_cfg4.npz"))
    N, C, H, W, layer, S, y0, x0, seed, M = (int(v) for v in g["geometry"])
    sx, sy = g["shiftx"].astype(np.int32), g["shifty"].astype(np.int32)
    frames = torch.empty(N * C * H * W, dtype=torch.int16, device="cuda")
    gpu_ctx.synth_fill(frames.data_ptr(), N, C, H, W, 0, H, seed, M)
    fv = frames.view(N, C, H, W)
    starts = [H // 8 - 32, 3 * H // 8 - 32, 5 * H // 8 - 32] if part == 0 else \
        [H // 8 + 96, 5 * H // 8 + 96, 7 * H // 8 + 96]
    jobs = [(c, j) for c in range(C) for j in _oracle_band_jobs(fv, starts, 64, M, C=c)]

    def oracle_bands():
        res = []
        for c, (b, lo, band) in jobs:
            rc, ref, _, rows = orc.stack_rejection(band, sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                                   max_thread=16, max_number_of_rows=16 * 24, row_counters=True)
            res.append((c, b, rc, ref[0, b - lo:b + 64 - lo].copy(), rows[0, b - lo:b + 64 - lo].sum(axis=0)))
        return res

    pool = ThreadPoolExecutor(1)
    fut = pool.submit(oracle_bands)
    out = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              max_thread=16, max_number_of_rows=H)
    gpu_ctx.stack_device(desc, frames.data_ptr(), C * H * W, H * W, out.data_ptr(), 0, H)
    assert gpu_ctx.stats().path == 1
    band_rej = {}
    ob = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    for b in starts:        # each band's counters from a band call of its own
        r, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), C * H * W, H * W, ob.data_ptr(), b, b + 64)
        band_rej[b] = r.copy()
    img = out.cpu().numpy().view(np.uint16).reshape(C, H, W)
    for c, b, rc, want, rows in fut.result():
        assert rc == 0
        bad = np.argwhere(img[c, b:b + 64] != want)
        assert bad.size == 0, f"channel {c} rows {b}..{b + 64}: {len(bad)} pixels differ, first {bad[:3].tolist()}"
        assert np.array_equal(band_rej[b][c], rows), (c, b, band_rej[b][c], rows)
    pool.shutdown()
    del frames, out, ob, fv
    _free()


@pytest.mark.parametrize("normalize", ["additive-scaling", "multiplicative-scaling"])
def test_cfg2_normalised_fma_load_whole_image(gpu_ctx, normalize):
    """configs[2]'s 512 x 4096^2 SIGMA (4, 3) stack normalised as bench.py's --normalize (the GUI
    defaults; coefficients as compute_normalization forms them, stacking.c:79-190): the histogram
    kernel's single-rounding load (admitted by k_norm_fma_check, norm_fma = 1) gives the same whole
    image and counters as a context held to the reference's roundings (SG_NORM_FMA=0, norm_fma = 0),
    and 3 row bands (top, middle, bottom) equal the oracle (stacking.c:1642-1651)"""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    frames, sx, sy, (N, H, W, M) = _sigma_cfg2(gpu_ctx)
    fv = frames.view(N, H, W)
    i = np.arange(N, dtype=np.float64)
    loc = 1000.0 + 0.6 * np.sin(0.37 * i)
    scl = 30.0 + 0.3 * np.cos(0.23 * i)
    scale = scl[0] / scl
    if normalize == "additive-scaling":
        mode, off, mul = sg.ADDITIVE_SCALING, scale * loc - loc[0], np.ones(N)
    else:
        mode, off, mul = sg.MULTIPLICATIVE_SCALING, np.zeros(N), loc[0] / loc
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=mode, offset=off, mul=mul, scale=scale, max_thread=16, max_number_of_rows=H)
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    outr = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rej, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    assert gpu_ctx.stats().norm_fma == 1, "the single-rounding load was not admitted"
    old = os.environ.get("SG_NORM_FMA")
    os.environ["SG_NORM_FMA"] = "0"
    try:
        ref_ctx = sg.Context()
    finally:
        if old is None:
            del os.environ["SG_NORM_FMA"]
        else:
            os.environ["SG_NORM_FMA"] = old
    try:
        rej_r, _ = ref_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, outr.data_ptr(), 0, H)
        assert ref_ctx.stats().norm_fma == 0
    finally:
        ref_ctx.close()
    assert torch.equal(out, outr), f"{normalize}: the fma load's image differs from the reference roundings'"
    assert np.array_equal(rej, rej_r), (rej, rej_r)
    R = 64
    starts = [0, H // 2, H - R]
    jobs = _oracle_band_jobs(fv, starts, R, M)

    def oracle_bands():
        res = []
        for b, lo, band in jobs:
            rc, ref, _, rows = orc.stack_rejection(band, sg.SIGMA, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                                   normalize=mode, offset=off, mul=mul, scale=scale, max_thread=16,
                                                   max_number_of_rows=16 * 24, row_counters=True)
            res.append((b, rc, ref[0, b - lo:b + R - lo].copy(), rows[0, b - lo:b + R - lo].sum(axis=0)))
        return res

    pool = ThreadPoolExecutor(1)
    fut = pool.submit(oracle_bands)
    img = out.cpu().numpy().view(np.uint16).reshape(H, W)
    band_rej = {}
    for b in starts:
        r, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, outr.data_ptr(), b, b + R)
        band_rej[b] = r.copy()
    for b, rc, want, rows in fut.result():
        assert rc == 0
        bad = np.argwhere(img[b:b + R] != want)
        assert bad.size == 0, f"{normalize} rows {b}..{b + R}: {len(bad)} pixels differ, first {bad[:3].tolist()}"
        assert np.array_equal(band_rej[b][0], rows), (b, band_rej[b][0], rows)
    pool.shutdown()
    del frames, out, outr, fv
    _free()
