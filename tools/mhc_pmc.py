"""Run the fused mHC kernel for the three backbone shapes (for rocprofv3 --pmc passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ManifoldHyperConnection  # noqa: E402
from hv_amd import manifold as MF  # noqa: E402

for D, T in [(32, 409600), (64, 409600), (128, 102400)]:
    m = ManifoldHyperConnection(D, expansion_rate=4).cuda().eval()
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    p = m.plan()
    with torch.no_grad():
        for _ in range(3):
            MF.mhc_apply(x, p)
torch.cuda.synchronize()
print("done")
