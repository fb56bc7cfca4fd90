"""Data-parallel gradient path of the trainer on CPU with gloo, world_size 2:
bucketed, hook-driven all-reduce must produce the rank-average of the per-rank gradients,
unused-parameter buckets must still be reduced, and buffer broadcast must make replicas
identical (DDP broadcast_buffers semantics)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "humanoid-vision-system_amd")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.mhc_like = torch.nn.Linear(32, 8)
        self.unused = torch.nn.Linear(4, 4)
        self.bn = torch.nn.BatchNorm1d(8)

    def forward(self, x):
        return self.bn(self.mhc_like(torch.relu(self.a(x))))


def _worker(rank, world, port, bucket_bytes, q):
    sys.path[:0] = [ROOT, PKG]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hv_amd.trainer import GradBuckets
        torch.manual_seed(0)
        net = Net()
        gb = GradBuckets(list(net.named_parameters()), bucket_bytes=bucket_bytes)
        res = {}
        for step in range(2):
            gb.zero()
            torch.manual_seed(100 + 10 * rank + step)
            x = torch.randn(12, 16)
            net(x).pow(2).sum().backward()
            gb.finish()
            # numpy copies travel by value: tensors would be passed as shared-memory fds that the
            # parent can only open while this process is alive (a race with its exit)
            res[step] = {n: p.grad.detach().clone().numpy() for n, p in net.named_parameters()}
        q.put((rank, res, len(gb.buckets)))
    finally:
        dist.destroy_process_group()


def _reference_grads(world):
    torch.manual_seed(0)
    net = Net()
    out = {}
    for step in range(2):
        acc = None
        for r in range(world):
            net.zero_grad()
            torch.manual_seed(100 + 10 * r + step)
            x = torch.randn(12, 16)
            net(x).pow(2).sum().backward()
            g = {n: (p.grad.clone() if p.grad is not None else torch.zeros_like(p)) for n, p in net.named_parameters()}
            acc = g if acc is None else {n: acc[n] + g[n] for n in acc}
        out[step] = {n: v / world for n, v in acc.items()}
    return out


@pytest.mark.parametrize("bucket_bytes", [64, 1 << 20])
def test_bucketed_allreduce_averages_gradients(bucket_bytes):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_bytes, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _reference_grads(world)
    for rank, res, nb in results:
        if bucket_bytes == 64:
            assert nb > 2          # several buckets exercised
        for step in (0, 1):
            for n, g in res[step].items():
                torch.testing.assert_close(torch.from_numpy(g), ref[step][n], rtol=1e-5, atol=1e-6)


def test_mhc_group_assignment():
    sys.path[:0] = [ROOT, PKG]
    from hv_amd.trainer import mhc_group
    assert mhc_group("backbone.stem.0.mhc.H_pre_raw") == 0
    assert mhc_group("vit_encoder.fusion_mhc.mlp.0.weight") == 0
    assert mhc_group("final_fusion.H_res_raw") == 0          # 'H_' in name
    assert mhc_group("backbone.stem.0.conv.weight") == 1
    assert mhc_group("detection_head.pred_heads.0.pred_conv.bias") == 1
