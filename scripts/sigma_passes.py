"""A/B helper: SIGMA pass counts per pixel on the histogram path, from a probe build of the
library (-DSGH_SIGMA_PASSES: the output image holds each pixel's pass count, the final pass that
removes nothing included; run with SG_LIB_PATH pointing at that build).  Workload: 1024 rows of
the bench's 512 x 4096 sequence, SIGMA (4, 3).  Pixels the literal replay writes afterwards
(early-break chains) show their stacked values (~1000), not counts: exclude values > 500."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sirilgpu as sg  # noqa: E402
import bench  # noqa: E402

N, H, W = 512, 1024, 4096
torch.cuda.set_device(0)
ctx = sg.Context([0])
frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
torch.cuda.synchronize()
ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, 16)
shx, shy = bench.synth_shifts_np(N, 0x5151, 16)
desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=shx, shifty=shy,
                          max_thread=8, max_number_of_rows=H)
ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
kms = ctx.stats().kernel_ms
torch.cuda.synchronize()
it = out.cpu().numpy().view(np.uint16).reshape(H, W).astype(np.int64)
it = np.where(it > 500, 0, it)          # pixels written by the literal replay, not counts
# SIGMA: a wave finishes 32 consecutive pixel columns col = 32 w + (lane >> 1) of the tile,
# column col = 64 g + l is image pixel x0 + 2 l + g (g = 0, 1): wave w takes lanes l of
# parity (col >> 6) -> waves 0, 1: even pixels 0..63 / 64..127 of the even set
nt = W // 128
t = it[:, : nt * 128].reshape(H, nt, 64, 2)            # [row][tile][l][g]
cols = t.transpose(0, 1, 3, 2).reshape(H, nt, 128)      # column index col = 64 g + l
waves = cols.reshape(-1, 32)                            # 32 columns per wave
wmax, wmean = waves.max(axis=1), waves.mean(axis=1)
print(f"kernel_ms {kms:.3f}; passes per pixel: mean {it.mean():.2f} p50 {np.median(it):.0f} "
      f"p90 {np.percentile(it, 90):.0f} p99 {np.percentile(it, 99):.0f} max {it.max()}")
print(f"per wave: max mean {wmax.mean():.2f} (p50 {np.median(wmax):.0f}, p90 {np.percentile(wmax, 90):.0f}); "
      f"lane mean {wmean.mean():.2f}; efficiency (lane mean / max) {wmean.sum() / wmax.sum():.3f}")
hist = np.bincount(np.minimum(it.ravel(), 20))
print("histogram of per-pixel counts (0..20+):", hist.tolist())
