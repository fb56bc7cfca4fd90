"""Is the training step host-bound?  Times the host-side enqueue of each HVTrainer.step (no
sync) against the wall time including the GPU drain, at base 640, B=16, bf16.
usage: python tools/train_hostbound.py [batch] [size]"""
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
S = int(sys.argv[2]) if len(sys.argv) > 2 else 640
dev = torch.device("cuda")
from hv_amd import _lib  # noqa: E402
for knob, fn in (("HV_TRAIN128", "hv_gemm_set_train128"), ("HV_STAGED_TRAIN", "hv_gemm_set_staged_train")):
    if os.environ.get(knob) is not None:
        getattr(_lib.lib(), fn)(int(os.environ[knob]))
        print(f"{knob}={os.environ[knob]}")
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": S, "verbose": False}).to(dev).train()
tr = HVTrainer(m)
x = torch.randn(B, 3, S, S, device=dev)
tg = [t.to(dev) for t in synthetic_targets(B, S, seed=1000)]
for _ in range(2):
    tr.step(x, tg)
torch.cuda.synchronize()
for i in range(4):
    t0 = time.perf_counter()
    tr.step(x, tg)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"step {i}: host enqueue {1e3 * (t1 - t0):7.2f} ms, wall {1e3 * (t2 - t0):7.2f} ms", flush=True)
# forward only / backward only split (host)
torch.cuda.synchronize()
t0 = time.perf_counter()
tr.model.train()
tr.grads.zero()
out = m(x, targets=tg, compute_loss=True)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
out["loss"]["total_loss"].backward()
t3 = time.perf_counter()
torch.cuda.synchronize()
t4 = time.perf_counter()
print(f"forward: host {1e3 * (t1 - t0):.2f} ms, gpu-drained {1e3 * (t2 - t0):.2f} ms; "
      f"backward: host {1e3 * (t3 - t2):.2f} ms, gpu-drained {1e3 * (t4 - t2):.2f} ms")
