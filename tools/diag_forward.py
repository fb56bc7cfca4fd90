"""Diagnostic: one tiny-config forward with a synchronise after every op (HV_SYNC_CHECK=1)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 224
tiny = (sys.argv[3] if len(sys.argv) > 3 else "tiny") == "tiny"
cfg = dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5) if tiny else {}
m = HybridVisionSystem(dict(cfg, precision=prec, verbose=False)).cuda().eval()
x = torch.randn(2, 3, size, size, device="cuda")
out = m(x)
torch.cuda.synchronize()
print("OK", {k: tuple(v.shape) for k, v in out["predictions"].items()})
