"""Batch-1 streaming latency profile: frozen hipGraph replay of the 640x640 bf16 forward
(config E), for rocprofv3 --kernel-trace --stats."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).cuda().eval()
if os.environ.get("HV_SET"):       # e.g. HV_SET="detect.LATERALS_BESIDE_VIT=False": hv_amd module switches
    import ast
    import importlib
    for kv in os.environ["HV_SET"].split(","):
        k, v = kv.split("=")
        mod, name = k.rsplit(".", 1)
        setattr(importlib.import_module("hv_amd." + mod), name, ast.literal_eval(v))
if os.environ.get("HV_OPTS"):      # e.g. HV_OPTS="branch_min_batch=1,mhc_tok=False"
    import ast
    m.set_options(**{k: ast.literal_eval(v) for k, v in (kv.split("=") for kv in os.environ["HV_OPTS"].split(","))})
m.freeze(not os.environ.get("HV_LAT_RECOMPUTE"))     # HV_LAT_RECOMPUTE=1: prep re-run per frame
x = torch.randn(1, 3, 640, 640, device="cuda")
with torch.no_grad():
    m(x)
    r = m.capture(x)
    for _ in range(5):
        r(x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        r(x)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
ts.sort()
print(f"{'recompute' if os.environ.get('HV_LAT_RECOMPUTE') else 'frozen'} B=1 p50 {ts[len(ts) // 2]:.3f} ms over {reps}")
