"""The headline workload at its full size (BASELINE configs[2]: SIGMA (4, 3) stack of 512
synthetic 4096 x 4096 frames with registration shifts, the bench's generator and shifts),
checked bit for bit against the C oracle on sampled row bands.

The oracle stacks a band of rows as a standalone image: the reference's y shift is a
translation with zero fill outside the frame (src/stacking/stacking.c:1550-1577), so output
rows [b, e) of the full image equal the oracle's rows of the band image [b - 16, e + 16)
(|shifty| <= 16) whenever that band lies inside the frame or shares the frame border.  Bands:
the top and bottom rows (out-of-frame zero fill) and a middle band.  At N = 512 the first
clipping pass never breaks early, so no pixel depends on the previous pixel's stale
rejected[] (the band's thread order cannot matter)."""
import os
import sys

import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_sigma_full_size_bands_match_oracle(gpu_ctx):
    import torch
    import bench
    N, H, W, M = 512, 4096, 4096, 16
    frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, M)
    sx, sy = bench.synth_shifts_np(N, 0x5151, M)
    assert int(np.abs(sy).max()) <= M
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              max_thread=16, max_number_of_rows=H)
    rej, _ = gpu_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    torch.cuda.synchronize()
    img = out.cpu().numpy().view(np.uint16).reshape(H, W)
    fr = frames.view(N, H, W)
    for b, e in [(0, 64), (2016, 2080), (H - 64, H)]:
        lo, hi = max(0, b - M), min(H, e + M)
        band = fr[:, lo:hi, :].cpu().numpy().view(np.uint16)[:, None]
        # 4 row blocks of >= 20 rows (max_number_of_rows / max_thread = 24): every block is
        # taller than the shifts, as the reference needs (its offset bug)
        rc, ref, _ = orc.stack_rejection(band, sg.SIGMA, sig=(4.0, 3.0), shiftx=sx, shifty=sy, max_thread=16,
                                         max_number_of_rows=16 * 24)
        assert rc == 0
        got, want = img[b:e], ref[0, b - lo:e - lo]
        bad = np.argwhere(got != want)
        assert bad.size == 0, f"rows {b}..{e}: {len(bad)} pixels differ, first {bad[:3].tolist()}"
    # the whole image: every pixel written, values in the synthetic range
    assert int(img.min()) > 0 and np.isfinite(img).all()


def test_winsorized_full_size_bands_match_oracle(gpu_ctx):
    """configs[4]'s frame size and rejection (256 frames of 6000 x 4000, WINSORIZED (4, 3)),
    one channel, sampled row bands against the oracle"""
    import torch
    import bench
    N, H, W, M = 256, 4000, 6000, 16
    frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x7777, M)
    sx, sy = bench.synth_shifts_np(N, 0x7777, M)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx,
                              shifty=sy, max_thread=16, max_number_of_rows=H)
    gpu_ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    torch.cuda.synchronize()
    img = out.cpu().numpy().view(np.uint16).reshape(H, W)
    fr = frames.view(N, H, W)
    for b, e in [(0, 64), (1968, 2032), (H - 64, H)]:
        lo, hi = max(0, b - M), min(H, e + M)
        band = fr[:, lo:hi, :].cpu().numpy().view(np.uint16)[:, None]
        rc, ref, _ = orc.stack_rejection(band, sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                         max_thread=16, max_number_of_rows=16 * 24)
        assert rc == 0
        got, want = img[b:e], ref[0, b - lo:e - lo]
        bad = np.argwhere(got != want)
        assert bad.size == 0, f"rows {b}..{e}: {len(bad)} pixels differ, first {bad[:3].tolist()}"
