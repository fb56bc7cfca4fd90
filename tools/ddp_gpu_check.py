"""2-rank data-parallel training check on ONE GPU (both ranks on cuda:0, gloo moves the
gradient buckets through host memory): after two HVTrainer steps on different per-rank
batches, every parameter must be bitwise identical across ranks (rank-0 broadcast at
construction + averaged gradients + identical optimizer), and the averaged gradient must
equal the mean of the per-rank local gradients.

usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
           --master-port 29511 tools/ddp_gpu_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda:0")
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402

torch.manual_seed(1234 + rank)            # different init per rank: the trainer must broadcast rank 0's
m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False,
                            precision="fp32")).to(dev).train()
for mod in m.modules():                   # deterministic: the check compares two backward passes
    if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
        mod.p = 0.0
tr = HVTrainer(m, lr=1e-3, bucket_mb=1)
B, S = 2, 64
torch.manual_seed(99 + rank)
x = torch.randn(B, 3, S, S, device=dev)
tg = [t.to(dev) for t in synthetic_targets(B, S, seed=3 + rank)]
# local gradient of this rank (no reduction) for the averaging check
tr.grads.zero()
hooks_world = tr.grads.world
tr.grads.world = 1                        # disable the hooks' reduction for one local backward
for h in tr.grads._hooks:
    h.remove()
out = m(x, targets=tg, compute_loss=True)
out["loss"]["total_loss"].backward()
# the local gradients in the flat buffer's layout (zero() leaves param.grad None, so without the
# hooks the backward stored them in param.grad, not in the flat views)
local = torch.zeros_like(tr.grads.flat)
for p in tr.grads.params:
    if p.grad is not None:
        o = tr.grads.offsets[id(p)]
        local[o:o + p.numel()] = p.grad.detach().float().reshape(-1)
tr.grads.world = hooks_world
with tr._on_stream():                     # the trainer's hooks live on its stream (HVTrainer.__init__)
    g = tr.grads
    g._hooks = [p.register_hook(g._flag_hook(i)) for i, p in enumerate(g.params)]
    g._hooks += [p.register_post_accumulate_grad_hook(g._on_grad) for p in g.params]
torch.manual_seed(7)
for step in range(2):
    loss = tr.step(x, tg)
    if step == 0:
        avg = tr.grads.flat.clone()
ref = local.clone()
dist.all_reduce(ref)
ref /= world
err = ((avg - ref).norm() / ref.norm()).item()
flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
other = flat.clone()
dist.broadcast(other, 0)
same = torch.equal(flat, other)
print(f"rank {rank}: loss {loss['total_loss'].item():.4f} avg-grad rel err {err:.2e} params identical {same}",
      flush=True)
ok = torch.tensor([1.0 if (same and err < 1e-4) else 0.0])
dist.all_reduce(ok)
dist.destroy_process_group()
sys.exit(0 if ok.item() == world else 1)
