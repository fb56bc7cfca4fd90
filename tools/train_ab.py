"""Same-process A/B of training-step options on the bench's training workload (base 640, B=16,
bf16, HVTrainer graph replay): model attributes toggled per arm, separate trainers and models,
arms interleaved.  usage: python tools/train_ab.py <attr> [batch] [steps]
  attr: a model attribute switched False (arm A) / True (arm B), e.g. hv_train_group_prep, or
        TF.<name>: a hv_amd.train_fn module switch (e.g. TF.EPILOGUE_COLSUM), or
        GV.<bits>: arm B runs with HVOptions.gemm_variant = bits (e.g. GV.0x80, 128x128 training tiles)
        WV.<bits>: arm B runs with HVOptions.wgrad_variant = bits (HV_WV_*)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402

attr = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
N = int(sys.argv[3]) if len(sys.argv) > 3 else 6
dev = torch.device("cuda")
x = torch.randn(B, 3, 640, 640, device=dev)
tg = [t.to(dev) for t in synthetic_targets(B, 640, seed=3)]
arms = {}
for val in (False, True):
    torch.manual_seed(0)
    m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).to(dev).train()
    if attr.startswith("TF."):            # a hv_amd.train_fn module switch, set around each arm's steps
        import hv_amd.train_fn as TF
        setattr(TF, attr[3:], val)
    elif attr.startswith("GV."):
        if val:
            m.set_options(gemm_variant=int(attr[3:], 0))
    elif attr.startswith("WV."):
        if val:
            m.set_options(wgrad_variant=int(attr[3:], 0))
    else:
        setattr(m, attr, val)
    arms[val] = HVTrainer(m, monitor_every=0, graph=True)
    for _ in range(3):
        arms[val].step(x, tg)
    torch.cuda.synchronize()
res = {False: [], True: []}
for rnd in range(3):
    for val in (False, True):
        tr = arms[val]
        if attr.startswith("TF."):
            setattr(TF, attr[3:], val)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            loss = tr.step(x, tg)
        torch.cuda.synchronize()
        res[val].append((time.perf_counter() - t0) / N * 1e3)
for val in (False, True):
    ts = sorted(res[val])
    print(f"{attr}={val}: median {ts[1]:.2f} ms/step ({B / ts[1] * 1e3:.1f} img/s) all {['%.2f' % t for t in res[val]]} "
          f"loss {float(arms[val].step(x, tg)['total_loss']):.3f}", flush=True)
