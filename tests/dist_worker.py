"""Worker of tests/test_dist_gloo.py (one rank; started as a subprocess):
python dist_worker.py RANK WORLD PORT IN.npz OUT.npz"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "siril-0.9_amd", "python"))

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle_numpy as onp  # noqa: E402
import sirilgpu_dist as sd  # noqa: E402


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    d = np.load(sys.argv[4], allow_pickle=False)
    frames, sx, sy, sig = d["frames"], d["sx"], d["sy"], tuple(float(v) for v in d["sig"])
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        H = frames.shape[2]

        def stack_band(b, e):
            out, rej = onp.stack_rejection_1thread(frames, 2, sig, sx, sy, rows=(b, e))
            return out[:, b:e], rej

        img, rej = sd.stack_sharded(stack_band, H, dist, rank, world)
        t = sd.max_time(0.5 + rank, dist)
        np.savez(sys.argv[5], img=img, rej=rej, t=np.array(t))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
