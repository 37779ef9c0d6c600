"""A/B probe: wave cycles per region of the Winsorized histogram finish on the configs[4]
workload (256 x 3 x 4000 x 6000).  Needs the probe build (-DSGH_WPROF, SG_LIB_PATH): the
finishing waves accumulate their region cycles in LDS (scripts sgh_wp) and add them into the
first u64 slots of the output buffer (outputs and redo list are not written in that build)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sirilgpu as sg  # noqa: E402
import bench  # noqa: E402

N, C, H, W = 256, 3, 4000, 6000
seed, M = 0x5EED, 16
torch.cuda.set_device(0)
ctx = sg.Context([0])
frames = torch.empty(N * C * H * W, dtype=torch.int16, device="cuda")
out = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
ctx.synth_fill(frames.data_ptr(), N, C, H, W, 0, H, seed, M)
sx, sy = bench.synth_shifts_np(N, seed, M)
desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                          max_thread=8, max_number_of_rows=H)
for it in range(3):
    out.zero_()
    torch.cuda.synchronize()
    ctx.stack_device(desc, frames.data_ptr(), C * H * W, H * W, out.data_ptr(), 0, H)
    torch.cuda.synchronize()
    kms = ctx.stats().kernel_ms
v = out.cpu().numpy().view(np.uint64)[:16].astype(np.float64)
nw = v[0]
names = ["prefix", "pass start (sigma, median)", "inner: before queries", "inner: queries",
         "inner: after queries", "clip pass", "tail (write, counts)"]
tot = v[1:8].sum()
print(f"kernel_ms {kms:.3f}  finishing waves {nw:.0f}  cycles per wave {tot / nw:.0f}")
for i, n in enumerate(names):
    print(f"  {n:28s} {v[1 + i] / nw:9.0f} cycles/wave  {100 * v[1 + i] / tot:5.1f} %")
print(f"  inner iterations per wave {v[8] / nw:.2f}, passes per wave {v[9] / nw:.2f}")
ev = ["query-loop bodies", "plain count queries (ambiguous thresholds)", "iterations with a slow threshold",
      "low growths", "high growths", "sigma-zero iterations"]
for i, n in enumerate(ev):
    print(f"  {n:44s} {v[10 + i] / nw:7.2f} per wave")
