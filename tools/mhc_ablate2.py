"""Ablation timing of the split-hidden fused mHC kernel (variants 3 / 4, D=128): which phase
dominates (diagnostic knob hv_mhc_fused_set_ablate; outputs are garbage when ablated)."""
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
lib.hv_mhc_fused_set_variant.argtypes = [ctypes.c_int]
D, T = 128, int(sys.argv[1]) if len(sys.argv) > 1 else 102400
m = ManifoldHyperConnection(D, expansion_rate=4).cuda().eval()
x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
p = m.plan()
names = {2048: "ret before GEMM3", 4096: "ret before LN", 0: "full", 1: "no weight DMA", 2: "no GEMM2", 4: "no GEMM1", 8: "no GEMM3", 6: "no GEMM1+2",
         7: "no DMA+GEMM1+2", 15: "all", 31: "all+no loop sync", 47: "all+no loop LDS reads",
         63: "all+no sync+reads", 16: "no loop sync only", 256: "return at entry", 512: "return after prologue",
         1024: "return after loop", 1025: "ret after loop, no DMA"}
for var in (4,):
    lib.hv_mhc_fused_set_variant(var)
    res = {k: [] for k in names}
    with torch.no_grad():
        for rep in range(5):
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
    for k, ts in res.items():
        print(f"variant {var} T={T} {names[k]:16s} {sorted(ts)[2] * 1e3:8.1f} us", flush=True)
lib.hv_mhc_fused_set_variant(0)
