"""Per-shape timing (HIP events) of every GEMM-family launch in one base-640 training step:
forward/backward training GEMMs, plain GEMMs/convs, conv dgrad, weight-gradient GEMMs.

usage: python tools/train_gemm_breakdown.py [batch]
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem, ops  # noqa: E402
from hv_amd import ops_train as OT  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda")
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).to(dev).train()
tr = HVTrainer(m, monitor_every=0)
x = torch.randn(B, 3, 640, 640, device=dev)
tg = [t.to(dev) for t in synthetic_targets(B, 640, seed=3)]
tr.step(x, tg)
torch.cuda.synchronize()

recs = []


def wrap(name, fn, shape_of):
    def f(*a, **k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn(*a, **k)
        e.record()
        recs.append((name,) + shape_of(a, k, out) + (s, e))
        return out
    return f


orig = {}
targets = [
    (ops, "gemm", lambda a, k, o: (a[0].shape[0], a[1].shape[0], a[1].shape[1])),
    (ops, "conv2d", lambda a, k, o: (o.shape[0] * o.shape[1] * o.shape[2], a[1].shape[0], a[1].shape[1])),
    (OT, "gemm_train", lambda a, k, o: (a[0].shape[0], a[1].shape[0], a[1].shape[1])),
    (OT, "conv_dgrad", lambda a, k, o: (o.shape[0] * o.shape[1] * o.shape[2], o.shape[3], a[1].shape[1])),
    (OT, "wgrad", lambda a, k, o: (a[0].shape[0], a[0].shape[1], a[1].shape[1])),
    (OT, "conv_wgrad", lambda a, k, o: (a[0].shape[0] * a[0].shape[1] * a[0].shape[2], o.shape[0], o.shape[1])),
]
import hv_amd.train_fn as TF  # noqa: E402
import hv_amd.train_model as TM  # noqa: E402
for mod, name, shp in targets:
    orig[(mod, name)] = getattr(mod, name)
    w = wrap(name, getattr(mod, name), shp)
    setattr(mod, name, w)
    for m2 in (TF, TM):
        if getattr(m2, name, None) is orig[(mod, name)]:
            setattr(m2, name, w)
tr.step(x, tg)
torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for name, M, N, K, s, e in recs:
    a = agg[(name, M, N, K)]
    a[0] += 1
    a[1] += s.elapsed_time(e)
    a[2] += 2.0 * M * N * K
tot = sum(v[1] for v in agg.values())
byk = collections.defaultdict(lambda: [0, 0.0, 0.0])
for (name, M, N, K), (n, ms, fl) in agg.items():
    byk[name][0] += n
    byk[name][1] += ms
    byk[name][2] += fl
print(f"GEMM-family total {tot:.1f} ms over {len(recs)} launches (B={B})")
for k, (n, ms, fl) in sorted(byk.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:<12}{n:>5} launches {ms:9.2f} ms {fl / (ms * 1e-3) / 1e12:8.1f} TF/s")
print(f"{'kind':<12}{'M/P':>9}{'N':>6}{'K':>6}{'n':>4}{'ms':>9}{'%':>6}{'TF/s':>8}")
for (name, M, N, K), (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:50]:
    print(f"{name:<12}{M:>9}{N:>6}{K:>6}{n:>4}{ms:>9.3f}{ms / tot * 100:>6.1f}{fl / (ms * 1e-3) / 1e12:>8.1f}")
