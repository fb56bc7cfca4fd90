"""bench.py's multi-GPU contract on CPU: `bench.py --gpus N` outside torchrun re-launches itself
as N ranks (torch.distributed.run, rendezvous on 127.0.0.1) and rank 0 alone prints ONE JSON
line carrying n_gpus = N (--dry-run skips the GPU work, keeps launcher + rendezvous +
max-over-ranks + report)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_gpus_flag_launches_n_ranks(n):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run", "--steps", "2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["ranks"] == list(range(n)) and rec["steps"] == 2
    assert rec["config"]["parallelism"] == f"replicas{n}"


def test_host_threads_respects_omp():
    sys.path.insert(0, ROOT)
    import bench
    old = os.environ.get("OMP_NUM_THREADS")
    try:
        os.environ["OMP_NUM_THREADS"] = "1"
        assert bench.host_threads() == 1
        os.environ.pop("OMP_NUM_THREADS")
        assert bench.host_threads() == len(os.sched_getaffinity(0))
    finally:
        if old is not None:
            os.environ["OMP_NUM_THREADS"] = old
