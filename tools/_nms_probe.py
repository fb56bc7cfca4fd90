import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch
from hv_amd import HybridVisionSystem, ops, _lib
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "verbose": False}).cuda().eval()
x = torch.randn(1, 3, 640, 640, device="cuda")
with torch.no_grad():
    dec = m(x)["decoded"]
plan = ops.NmsPlan(dec, 0.25, 0.45, 100)
L = _lib.lib()
h = (ctypes.c_longlong * (2 * 8 * 48))()
for it in range(3):
    ctypes.memset(h, 0, ctypes.sizeof(h))
    plan.run(); torch.cuda.synchronize()
    L.hv_nms_debug_times(h)
    for K, nb in ((0, 3), (1, 1)):
        for b in range(nb):
            t = [h[(K * 8 + b) * 48 + k] for k in range(48)]
            base = t[0]
            rel = {k: round(((v & ((1 << 62) - 1)) - base) * 0.01, 2) for k, v in enumerate(t) if v}
            lv = {k - 8: (rel[k], "L" if t[k] >> 62 else "G") for k in sorted(rel) if k >= 8}
            print(f"it{it} K{K} seg{b}: stamps {[(k, rel[k]) for k in sorted(rel) if k < 8]}")
            print(f"    last={t[46]} kept={t[47]}"); print(f"    levels(depth: t us): {sorted(lv.items(), key=lambda kv: -kv[0])}")
print("kept", plan.count.tolist())
