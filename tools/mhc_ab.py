"""A/B the fused mHC kernel variants (per-call HV_MV_* shapes) against the unfused GEMM chain at
in-model shapes (B=16).  usage: python tools/mhc_ab.py [D:T[:expansion] ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ManifoldHyperConnection, _lib  # noqa: E402
from hv_amd import manifold as MF  # noqa: E402
from hv_amd.runtime import HVOptions, RunCtx, use_ctx  # noqa: E402

shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[1:]] or \
    [(32, 1638400), (64, 409600), (128, 102400), (128, 25600)]


def timed(fn, n=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


W = _lib.MV_WIDE
VARIANTS = [int(v) for v in os.environ.get("HV_MHC_VARIANTS", "0,1,2,5,6").split(",")]
CASES = {"unfused": HVOptions(use_fused_mhc=False)}
CASES.update({f"fused_v{v}": HVOptions(mhc_variant=W | v) for v in VARIANTS})

for shp in shapes:
    D, T, ex = shp if len(shp) == 3 else (*shp, 4)
    m = ManifoldHyperConnection(D, expansion_rate=ex).cuda().eval()
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    p = m.plan()
    Hd = ex * D
    fl = 2.0 * T * (D * 2 * Hd + 2 * Hd * Hd + (Hd + D) * D)
    res = {k: [] for k in CASES}
    with torch.no_grad():
        with use_ctx(RunCtx(dtype=torch.bfloat16, opts=CASES["unfused"])):
            ref = MF.mhc_apply(x, p).float()
        for rep in range(5):
            for k, o in CASES.items():
                with use_ctx(RunCtx(dtype=torch.bfloat16, opts=o)):
                    if rep == 0:
                        y = MF.mhc_apply(x, p).float()
                        print(f"D={D} T={T} {k}: rel err vs unfused {((y - ref).norm() / ref.norm()).item():.2e}",
                              flush=True)
                    res[k].append(timed(lambda: MF.mhc_apply(x, p)))
    for k, ts in res.items():
        t = sorted(ts)[len(ts) // 2]
        print(f"mhc D={D:4d} T={T:8d} {k:9s}: {t:.3f} ms {fl / t / 1e9:7.1f} TF/s", flush=True)
