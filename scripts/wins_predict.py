"""A/B helper: does a pixel's zero / 65535 count predict its Winsorize inner-iteration count?
Runs the probe builds lib_witer (-DSGH_WINS_ITERS: iterations per pixel) and lib_wfeat
(-DSGH_WINS_FEAT: zeros << 8 | 65535s) on scripts/wins_iters.py's workload and prints the
mean iterations per feature bucket and the finish cost (sum over waves of the max iteration
count of their 64 pixels) for the present even / odd split, for a split that puts the
predicted-slow pixels of a tile together, and for an ideal split (sorted by true count)."""
import ctypes
import os
import subprocess
import sys
import json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = {k: os.path.join(ROOT, "siril-0.9_amd", f"lib_{k}", "libsirilgpu.so") for k in ("witer", "wfeat")}

if len(sys.argv) > 1:     # child: one library, saves the image
    os.environ["SG_LIB_PATH"] = LIBS[sys.argv[1]]
    sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import sirilgpu as sg
    import bench
    N, H, W = 256, 1000, 6000
    torch.cuda.set_device(0)
    ctx = sg.Context([0])
    frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
    out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, 16)
    shx, shy = bench.synth_shifts_np(N, 0x5151, 16)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.WINSORIZED, sig=(4.0, 3.0), shiftx=shx, shifty=shy,
                              max_thread=8, max_number_of_rows=H)
    ctx.stack_device(desc, frames.data_ptr(), H * W, H * W, out.data_ptr(), 0, H)
    torch.cuda.synchronize()
    np.save(f"/tmp/wp_{sys.argv[1]}.npy", out.cpu().numpy().view(np.uint16).reshape(H, W))
    sys.exit(0)

import numpy as np
for k in LIBS:
    subprocess.run([sys.executable, __file__, k], check=True)
it = np.load("/tmp/wp_witer.npy").astype(np.int64)
ft = np.load("/tmp/wp_wfeat.npy").astype(np.int64)
nz, ns = ft >> 8, ft & 255
H, W = it.shape
print(f"iterations: mean {it.mean():.2f}")
for name, f in (("65535s", ns), ("zeros", nz)):
    print(name, "bucket: count, mean iterations")
    for b in range(0, 6):
        m = (f == b) if b < 5 else (f >= 5)
        if m.any():
            print(f"  {b}{'+' if b == 5 else ''}: {m.sum():8d} {it[m].mean():6.2f}")
nt = W // 128
t = it[:, :nt * 128].reshape(H * nt, 128)        # [tile][x - x0]
pred = ((ns >= 1) | (nz >= 1))[:, :nt * 128].reshape(H * nt, 128)
cur = t[:, 0::2].max(1) + t[:, 1::2].max(1)
order = np.argsort(~pred, axis=1, kind="stable")
tp = np.take_along_axis(t, order, 1)
prd = tp[:, :64].max(1) + tp[:, 64:].max(1)
ts = np.sort(t, axis=1)
ideal = ts[:, :64].max(1) + ts[:, 64:].max(1)
print(f"finish cost (sum of wave maxima per tile): even/odd {cur.mean():.2f}, predicted-slow first {prd.mean():.2f}, "
      f"ideal {ideal.mean():.2f}; predicted slow per tile {pred.sum(1).mean():.1f}")
for thr in (1, 2, 3):
    pr2 = ((ns >= thr) | (nz >= thr))[:, :nt * 128].reshape(H * nt, 128)
    o2 = np.argsort(~pr2, axis=1, kind="stable")
    t2 = np.take_along_axis(t, o2, 1)
    print(f"  threshold {thr}: {(t2[:, :64].max(1) + t2[:, 64:].max(1)).mean():.2f} (slow per tile {pr2.sum(1).mean():.1f})")
