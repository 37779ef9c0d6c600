"""A/B helper: per-tile timeline of k_stack_hist with 256-pixel tiles (SG_HIST_DBG=11:
s_memrealtime stamps at entry, after the build barrier, at the end of wave 0's finish and
of the last wave's finish, u64 [tile][4] in the output buffer) over the bench workload."""
import os
import sys
os.environ["SG_HIST_DBG"] = "11"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sirilgpu as sg  # noqa: E402
import bench  # noqa: E402

N, H, W = 512, 4096, 4096
torch.cuda.set_device(0)
ctx = sg.Context([0])
frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
torch.cuda.synchronize()
ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, 16)
shx, shy = bench.synth_shifts_np(N, 0x5151, 16)
desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=shx, shifty=shy,
                          max_thread=8, max_number_of_rows=H)
for _ in range(3):
    ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    kms = ctx.stats().kernel_ms
torch.cuda.synchronize()
nb = H * (W // 256)  # 256-pixel tiles (SG_HIST_NI=2)
raw = out.cpu().numpy().view(np.uint64)[: nb * 32].reshape(nb, 32).astype(np.int64)
t = raw[:, :4]
wv = raw[:, 4:28].reshape(nb, 8, 3)
t0, t1, t2, t3 = (t[:, i] for i in range(4))
ok = (t1 >= t0) & (t2 >= t1) & (t3 >= t2) & (t0 > 0)
print("kernel_ms", round(kms, 3), "tiles", nb, "valid", int(ok.sum()))
t0, t1, t2, t3 = t0[ok], t1[ok], t2[ok], t3[ok]
wv = wv[ok]
act = wv[:, :, 1] > 0          # waves that ran the finish
pre, loop = wv[:, :, 0][act], wv[:, :, 1][act]
pmax, psum = (wv[:, :, 2][act] & 0xFFFF), (wv[:, :, 2][act] >> 16)
print(f"finish per wave (core cycles): prefix p50 {np.median(pre):.0f} mean {pre.mean():.0f}; pass loop p50 "
      f"{np.median(loop):.0f} mean {loop.mean():.0f} p90 {np.percentile(loop, 90):.0f}")
print(f"passes per wave: max p50 {np.median(pmax):.0f} mean {pmax.mean():.2f}; lane-mean {psum.mean() / 64:.2f}; "
      f"cycles per max-pass {loop.sum() / max(pmax.sum(), 1):.0f}")
us = 0.01          # 100 MHz ticks -> us
span = (t3.max() - t0.min()) * us
for name, v in [("build (entry -> barrier)", t1 - t0), ("finish wave 0", t2 - t1), ("finish all waves", t3 - t1),
                ("tile total", t3 - t0)]:
    v = v * us
    print(f"{name:26s} mean {v.mean():7.2f} us  p10 {np.percentile(v, 10):7.2f}  p50 {np.median(v):7.2f}  "
          f"p90 {np.percentile(v, 90):7.2f}  max {v.max():7.2f}")
busy = ((t3 - t0) * us).sum()
print(f"span {span:.1f} us; sum of tile lifetimes / span = {busy / span:.1f} tiles resident on average "
      f"(512 slots = 2 per CU); finish share of tile lifetime {((t3 - t1).sum() / (t3 - t0).sum()):.3f}")
# resident tiles over time, and how many of them are in their finish
grid = np.linspace(t0.min(), t3.max(), 41)
for g in grid[1:-1:4]:
    res = ((t0 <= g) & (t3 > g)).sum()
    fin = ((t1 <= g) & (t3 > g)).sum()
    print(f"  t={(g - t0.min()) * us:7.1f} us resident {res:4d} in finish {fin:4d}")
