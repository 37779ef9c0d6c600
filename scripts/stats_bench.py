"""Normalisation statistics at the bench scale: IKSS location / scale of 512 synthetic
4096x4096 frames on the device (sg_frame_stats_ikss_device), the oracle's statistics()
restatement timed on one frame beside it, and the device result checked against it."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    torch.zeros(1, device="cuda")
    import sirilgpu as sg
    import oracle_lib as orc
    N, H, W = int(os.environ.get("N", 512)), 4096, 4096
    ctx = sg.Context()
    frames = torch.empty(N * H * W, dtype=torch.int16, device="cuda")
    ctx.synth_fill(frames.data_ptr(), N, 1, H, W, 0, H, 0x5151, 16)
    rc, loc, scl = ctx.frame_stats_ikss(frames.data_ptr(), 2, 1, H, W)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc, loc, scl = ctx.frame_stats_ikss(frames.data_ptr(), N, 1, H, W)
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t0
    f0 = frames[: H * W].cpu().numpy().view(np.uint16).reshape(1, H, W)
    t0 = time.perf_counter()
    orc_rc, l0, s0 = orc.statistics_ikss(f0)
    cpu_s = time.perf_counter() - t0
    print(json.dumps({"frames": N, "size": [H, W], "gpu_ms": round(gpu_s * 1e3, 2), "rc": rc,
                      "gpu_frames_per_s": round(N / gpu_s, 1), "cpu_oracle_s_per_frame": round(cpu_s, 3),
                      "cpu_threads": 1, "frame0": [loc[0], scl[0]], "oracle_frame0": [l0, s0],
                      "bit_exact_frame0": bool(loc[0] == l0 and scl[0] == s0)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
