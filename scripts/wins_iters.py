"""A/B helper: Winsorize inner-iteration counts per pixel on the histogram path, from a probe
build of the library (-DSGH_WINS_ITERS: the output image holds each pixel's inner iteration
count; run with SG_LIB_PATH pointing at that build).  Workload: one 6000 x 1000 channel of 256
synthetic frames with the bench's shifts, WINSORIZED (4, 3).  A wave finishes the even or the
odd pixels of a 128-pixel tile (64 lanes), so its loop runs the maximum over those 64."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sirilgpu as sg  # noqa: E402
import bench  # noqa: E402

N, H, W = 256, 1000, 6000
torch.cuda.set_device(0)
ctx = sg.Context([0])
frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
torch.cuda.synchronize()
ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, 16)
shx, shy = bench.synth_shifts_np(N, 0x5151, 16)
desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=shx, shifty=shy,
                          max_thread=8, max_number_of_rows=H)
ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
kms = ctx.stats().kernel_ms
torch.cuda.synchronize()
it = out.cpu().numpy().view(np.uint16).reshape(H, W).astype(np.int64)
nt = W // 128
tiles = it[:, : nt * 128].reshape(H, nt, 64, 2)        # [row][tile][lane][parity]
waves = tiles.transpose(0, 1, 3, 2).reshape(-1, 64)    # one row per wave (64 pixels)
wmax, wmean = waves.max(axis=1), waves.mean(axis=1)
print(f"kernel_ms {kms:.3f}; inner iterations per pixel: mean {it.mean():.2f} p50 {np.median(it):.0f} "
      f"p90 {np.percentile(it, 90):.0f} p99 {np.percentile(it, 99):.0f} max {it.max()}")
print(f"per wave: max mean {wmax.mean():.2f} (p50 {np.median(wmax):.0f}, p90 {np.percentile(wmax, 90):.0f}); "
      f"lane mean {wmean.mean():.2f}; efficiency (lane mean / max) {wmean.sum() / wmax.sum():.3f}")
hist = np.bincount(np.minimum(it.ravel(), 40))
print("histogram of per-pixel counts (0..40+):", hist.tolist())
