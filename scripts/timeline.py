"""A/B helper: per-block timeline of k_stack_hist (SG_HIST_DBG=11, s_memtime stamps written
into the output buffer) over the bench workload."""
import os, sys
os.environ["SG_HIST_DBG"] = "11"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import sirilgpu as sg
import bench

N, H, W = 512, 4096, 4096
ctx = sg.Context([0])
frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, 16)
shx, shy = bench.synth_shifts_np(N, 0x5151, 16)
desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(4.0, 3.0), shiftx=shx, shifty=shy,
                          max_thread=8, max_number_of_rows=H)
for _ in range(2):
    ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
torch.cuda.synchronize()
nb = H * W // 128
t = out.cpu().numpy().view(np.uint64)[: nb * 8].reshape(nb, 8).astype(np.int64)
start, bar1, bend, bar2, f0, f1 = (t[:, i] for i in range(6))
ok = (bar1 > start) & (f0 > bar2)
print("blocks", nb, "valid", ok.sum())
def q(name, v):
    v = v[ok]
    print(f"{name:12s} mean {v.mean():9.0f}  p10 {np.percentile(v,10):9.0f}  p50 {np.percentile(v,50):9.0f}  p90 {np.percentile(v,90):9.0f}")
q("startup", bar1 - start)
q("build", bend - bar1)
q("barrier2", bar2 - bend)
q("finish_w0", f0 - bar2)
q("finish_w1", f1 - bar2)
q("lifetime", np.maximum(f0, f1) - start)
hw = t[:, 6]
# HW_ID (gfx9): wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]
cu = (hw >> 8) & 15; se = (hw >> 13) & 7; sh = (hw >> 12) & 1
key = se * 32 + sh * 16 + cu
print("distinct (se,sh,cu) ids:", len(np.unique(key)))
# concurrency estimate on one XCD-local clock: sum of lifetimes / kernel span per id
xcd = np.arange(nb) & 7
for x in range(2):
    m = ok & (xcd == x)
    span = t[m, 4].max() - t[m, 0].min()
    busy = (np.maximum(t[m, 4], t[m, 5]) - t[m, 0]).sum()
    print(f"xcd {x}: span {span} cycles, avg concurrent blocks per CU {busy / span / 32:.2f}")
ctx.close()
