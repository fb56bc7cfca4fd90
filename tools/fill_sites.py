"""Where the small fills / copies of a training step come from: one base-config training step
(after two warm-up steps) under torch.profiler (CPU activity, Python stacks); every aten fill /
zero / copy op is grouped by the innermost hv_amd frames of its stack.

usage: python tools/fill_sites.py [batch] [size] > out.txt
"""
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
S = int(sys.argv[2]) if len(sys.argv) > 2 else 640
dev = torch.device("cuda")
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": S, "precision": "bf16", "verbose": False}).to(dev).train()
tr = HVTrainer(m, monitor_every=0)
x = torch.randn(B, 3, S, S, device=dev)
tg = [t.to(dev) for t in synthetic_targets(B, S, seed=3)]
for _ in range(2):
    tr.step(x, tg)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    tr.step(x, tg)
    torch.cuda.synchronize()

ops = ("aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::copy_", "aten::new_zeros",
       "aten::_to_copy", "aten::add_", "aten::div_", "aten::mul_")
sites, totals = Counter(), Counter()
for ev in prof.events():
    if ev.name not in ops:
        continue
    totals[ev.name] += 1
    st = [f for f in (ev.stack or []) if "hv_amd" in f or "tools/" in f]
    sites[(ev.name, " < ".join(s.split("hv_amd/")[-1] for s in st[:3]) or "(engine / no hv frame)")] += 1
print("per-step op counts:", dict(totals))
for (name, where), c in sites.most_common(60):
    print(f"{c:6d}  {name:18s} {where}")
