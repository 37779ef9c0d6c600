"""A/B helper: distribution of sigma-clip pass counts of the histogram path (SG_HIST_DBG=7)
over the bench workload, per pixel and per 64-pixel wave (the wave runs its slowest lane)."""
import os, sys
os.environ["SG_HIST_DBG"] = "7"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
import numpy as np
import torch
import sirilgpu as sg

N, H, W = 512, 4096, 4096
ctx = sg.Context([0])
frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
out = torch.empty(H * W, dtype=torch.int16, device="cuda")
ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, 16)
sys.path.insert(0, ROOT)
import bench
shx, shy = bench.synth_shifts_np(N, 0x5151, 16)
desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=shx, shifty=shy,
                          max_thread=8, max_number_of_rows=H)
ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
torch.cuda.synchronize()
o = out.cpu().numpy().view(np.uint16).reshape(H, W)
# tile: 128 px, lanes own pixels 2l (wave 0) and 2l+1 (wave 1)
px = o[:, :4096].reshape(H, 32, 64, 2)
ok = px < 100
print("pixel passes histogram:", np.bincount(np.where(ok, px, 0).ravel())[:16])
wmax = np.where(ok, px, 0).max(axis=2)
print("wave-max passes histogram:", np.bincount(wmax.ravel())[:16])
print("mean pixel passes", px[ok].mean(), "mean wave max", wmax.mean())
ctx.close()
