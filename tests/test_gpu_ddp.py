"""Two data-parallel ranks on ONE GPU (gloo moves the gradient buckets through host memory; RCCL
needs distinct devices): HVTrainer's device-side DDP path -- rank-0 broadcast at construction,
loss pre-scaling, bucketed all-reduce from the hooks, device 'received' flags, lagged bucket
agreement, clip + AdamW -- leaves the replicas bitwise identical and the averaged gradient equal
to the mean of the per-rank local gradients (tools/ddp_gpu_check.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_ddp_training_on_one_gpu(gpu_device):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(ROOT, "tools", "ddp_gpu_check.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("params identical True") == 2
