"""Worker of tests/test_dist_gloo.py::test_register_sharding_gloo (one rank, a subprocess):
python dist_reg_worker.py RANK WORLD PORT IN.npz OUT.npz.  The per-shard registration is the
C oracle (test infrastructure): shifts of the shard's frames, raw QualityEstimate values."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "siril-0.9_amd", "python"))

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle_lib as orc  # noqa: E402
import sirilgpu_dist as sd  # noqa: E402


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    d = np.load(sys.argv[4], allow_pickle=False)
    sel, ref, inc = d["sel"], int(d["ref"]), d["inc"]
    included = None if inc.size == 0 else inc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = sel.shape[0]

        def register_part(mine):
            sx, sy, _ = orc.register_dft(sel, ref_image=ref, included=mine)
            q = np.zeros(n, dtype=np.float64)
            q[ref] = orc.quality(sel[ref])
            for f in range(n):
                if mine[f] and f != ref:
                    q[f] = orc.quality(sel[f])
            return sx, sy, q

        gx, gy, gq = sd.register_sharded(register_part, n, ref, included, dist, rank, world)
        np.savez(sys.argv[5], sx=gx, sy=gy, q=gq)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
