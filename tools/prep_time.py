"""Per-forward coefficient / weight prep of the bench model (base 640 bf16): the grouped
PrepProgram run alone, 30 times, for rocprofv3 --kernel-trace --stats (k_pg1..4, k_wprep, sk_*)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd.runtime import RunCtx  # noqa: E402

torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).cuda().eval()
x = torch.randn(2, 3, 640, 640, device="cuda")
with torch.no_grad():
    m(x)
    m(x)
    p = m._sk_cache["program"]
    ctx = RunCtx(dtype=torch.bfloat16)
    torch.cuda.synchronize()
    for _ in range(30):
        p.run(ctx)
    torch.cuda.synchronize()
print("ok", type(p).__name__)
