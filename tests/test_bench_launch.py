"""bench.py --gpus N: without a launcher it starts N ranks itself (torch.distributed.run, child
processes, before any GPU call); under a launcher WORLD_SIZE must equal --gpus.  CPU only: the
children stop at SG_BENCH_LAUNCH_PROBE before touching a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    env.update(kw)
    return env


def test_self_launch_starts_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--steps", "1"], env=_env(SG_BENCH_LAUNCH_PROBE="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2]
    assert all(x["world"] == 3 and x["gpus"] == 3 for x in lines)


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=_env(WORLD_SIZE="2", RANK="0",
                       SG_BENCH_LAUNCH_PROBE="1"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=_env(SG_BENCH_LAUNCH_PROBE="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"rank": 0, "world": 1, "gpus": 1}
