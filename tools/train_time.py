"""Training-step time of the bench's training workload (base 640, bf16, HVTrainer graph replay)
in one process: for cross-process A/Bs of knobs read once per process (e.g. HV_COLRED_CAP).
usage: python tools/train_time.py [batch] [steps]  -> one line 'median ms/step'"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N = int(sys.argv[2]) if len(sys.argv) > 2 else 6
dev = torch.device("cuda")
x = torch.randn(B, 3, 640, 640, device=dev)
tg = [t.to(dev) for t in synthetic_targets(B, 640, seed=3)]
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).to(dev).train()
tr = HVTrainer(m, monitor_every=0, graph=True)
for _ in range(3):
    tr.step(x, tg)
ts = []
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        tr.step(x, tg)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) / N * 1e3)
ts.sort()
print(f"{os.environ.get('HV_COLRED_CAP', '-')}: median {ts[1]:.2f} ms/step ({B / ts[1] * 1e3:.1f} img/s) all "
      f"{['%.2f' % t for t in ts]}", flush=True)
