"""Time the fused mHC kernel variants (tile / occupancy) at the backbone shapes, interleaved."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ManifoldHyperConnection, _lib  # noqa: E402
from hv_amd import manifold as MF  # noqa: E402

lib = _lib.lib()
lib.hv_mhc_fused_set_variant.argtypes = [ctypes.c_int]
for D, T in [(32, 1638400), (64, 1638400), (64, 409600), (128, 102400)]:
    m = ManifoldHyperConnection(D, expansion_rate=4).cuda().eval()
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    p = m.plan()
    Hd = 4 * D
    fl = 2.0 * T * (D * 2 * Hd + 2 * Hd * Hd + (Hd + D) * D)
    res = {v: [] for v in (0, 1)}
    with torch.no_grad():
        MF.USE_FUSED = False
        ref = MF.mhc_apply(x, p).float()
        MF.USE_FUSED = True
        for rep in range(5):
            for v in res:
                lib.hv_mhc_fused_set_variant(v)
                y = MF.mhc_apply(x, p)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    MF.mhc_apply(x, p)
                e.record()
                torch.cuda.synchronize()
                res[v].append(s.elapsed_time(e) / 5)
                if rep == 0:
                    err = ((y.float() - ref).norm() / ref.norm()).item()
                    print(f"D={D} T={T} variant {v}: rel err vs unfused {err:.2e}")
    lib.hv_mhc_fused_set_variant(0)
    for v, ts in res.items():
        t = sorted(ts)[len(ts) // 2]
        print(f"mhc D={D:4d} T={T:8d} variant {v}: {t:.3f} ms {fl / t / 1e9:7.1f} TF/s")
