"""Ablation timing of the fused mHC kernel (D=64, T=409600): which phase dominates."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ManifoldHyperConnection, _lib  # noqa: E402
from hv_amd import manifold as MF  # noqa: E402

lib = _lib.lib()
lib.hv_mhc_fused_set_ablate.argtypes = [ctypes.c_int]
D, T = 64, 409600
m = ManifoldHyperConnection(D, expansion_rate=4).cuda().eval()
x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
p = m.plan()
names = {0: "full", 1: "no GELU", 2: "no weight prefetch", 4: "no chunk barrier", 8: "no GEMM2", 16: "no GEMM1",
         24: "no GEMM1+GEMM2", 31: "all ablated"}
res = {k: [] for k in names}
with torch.no_grad():
    for rep in range(6):
        for k in names:
            lib.hv_mhc_fused_set_ablate(k)
            for _ in range(2):
                MF.mhc_apply(x, p)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                MF.mhc_apply(x, p)
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) / 5)
lib.hv_mhc_fused_set_ablate(0)
for k, n in names.items():
    v = sorted(res[k])
    print(f"{n:22s} {v[len(v) // 2]:.3f} ms")
