"""Per-shape GEMM/conv timing of one base-640 forward (HIP events around every launch).

usage: python tools/gemm_breakdown.py [batch] [size] [precision]
"""
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
S = int(sys.argv[2]) if len(sys.argv) > 2 else 640
P = sys.argv[3] if len(sys.argv) > 3 else "bf16"

m = HybridVisionSystem({"precision": P, "verbose": False}).cuda().eval()
# one stream: HIP events around a launch time that launch only when nothing runs beside it
m.set_options(branch_min_batch=1 << 30, prep_overlap_min_batch=1 << 30, gemm_variant=int(os.environ.get("HV_GEMM_VARIANT", "0"), 0))
x = torch.randn(B, 3, S, S, device="cuda")
with torch.no_grad():
    m(x)
    m(x)
torch.cuda.synchronize()

recs = []
g0, c0 = ops.gemm, ops.conv2d


def gemm(a, b, **kw):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    out = g0(a, b, **kw)
    e.record()
    tag = "gemm" + ("+ln" if kw.get("a_mean") is not None else "") + ("+cat" if kw.get("a2") is not None else "")
    recs.append((tag, a.shape[0], b.shape[0], b.shape[1], s, e))
    return out


def conv2d(x, w, k, stride, pad, **kw):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    out = c0(x, w, k, stride, pad, **kw)
    e.record()
    recs.append((f"conv{k}x{k}s{stride}", out.shape[0] * out.shape[1] * out.shape[2], w.shape[0], w.shape[1], s, e))
    return out


OTHER = ("mhc_fused", "mhc_prep", "cast", "row_stats", "layernorm", "rmsnorm", "sinkhorn", "channel_mean",
         "se_mlp", "scale_residual", "upsample_add", "add_scaled", "add_rowvec", "attention", "gather_rows",
         "yolo_decode", "conv_weight_prep", "bn_fold", "gemv", "maxpool2x2", "nchw_to_nhwc", "vit_tokens")
orig = {n: getattr(ops, n) for n in OTHER if hasattr(ops, n)}


def wrap(name, fn):
    def f(*a, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn(*a, **kw)
        e.record()
        t = next((x for x in a if isinstance(x, torch.Tensor)), None)
        shp = tuple(t.shape) if t is not None else ()
        if name == "mhc_fused":
            shp = (a[0].shape[0], a[0].shape[1], a[3].shape[0])
        recs.append((name, shp, 0, 0, s, e))
        return out
    return f


for n, fn in orig.items():
    setattr(ops, n, wrap(n, fn))
import hv_amd.manifold as MF  # noqa: E402
import hv_amd.layers as LY  # noqa: E402
for mod in (MF, LY):
    for n in orig:
        if hasattr(mod, n):
            setattr(mod, n, getattr(ops, n))
ops.gemm, ops.conv2d = gemm, conv2d
with torch.no_grad():
    t0 = time.perf_counter()
    m(x)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
ops.gemm, ops.conv2d = g0, c0
for n, fn in orig.items():
    setattr(ops, n, fn)

agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
byop = collections.defaultdict(lambda: [0, 0.0])
for tag, M, N, K, s, e in recs:
    ms = s.elapsed_time(e)
    byop[tag.split("+")[0] if tag.startswith("gemm") else tag][0] += 1
    byop[tag.split("+")[0] if tag.startswith("gemm") else tag][1] += ms
    if not isinstance(M, int):
        continue
    a = agg[(tag, M, N, K)]
    a[0] += 1
    a[1] += ms
    a[2] += 2.0 * M * N * K
print("per-op totals (HIP events, eager):")
for k, (n, ms) in sorted(byop.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:<18}{n:>5} launches {ms:8.3f} ms")
fz = collections.defaultdict(lambda: [0, 0.0])
for tag, M, N, K, s, e in recs:
    if tag == "mhc_fused":
        fz[M][0] += 1
        fz[M][1] += s.elapsed_time(e)
for (T, D, Hd), (n, ms) in sorted(fz.items()):
    fl = 2.0 * T * (2 * D * Hd + 2 * Hd * Hd + (Hd + D) * D) * n
    print(f"  mhc_fused T={T:8d} D={D:4d} Hd={Hd:4d} n={n:3d} {ms:8.3f} ms {fl / (ms * 1e-3) / 1e12:7.1f} TF/s")
tot = sum(v[1] for v in agg.values())
print(f"forward wall {wall:.2f} ms; GEMM/conv total {tot:.2f} ms over {len(recs)} launches")
print(f"{'kind':<14}{'M':>9}{'N':>6}{'K':>6}{'n':>4}{'ms':>9}{'%':>6}{'TF/s':>8}")
for (tag, M, N, K), (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
    print(f"{tag:<14}{M:>9}{N:>6}{K:>6}{n:>4}{ms:>9.3f}{ms / tot * 100:>6.1f}{fl / (ms * 1e-3) / 1e12:>8.1f}")
