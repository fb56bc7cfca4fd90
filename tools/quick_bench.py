"""Graph-replay step time of the bench workload (base 640^2, B=16, bf16) for same-box A/Bs of two
builds: run it alternately with HV_LIB_PATH pointing at each libhvs.so.
usage: python tools/quick_bench.py [tag]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402

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
x = torch.randn(16, 3, 640, 640, device="cuda")
with torch.no_grad():
    m(x)
    r = m.capture(x)
    for _ in range(3):
        r.graph.replay()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            r.graph.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / 10 * 1e3)
ts.sort()
print(f"{sys.argv[1] if len(sys.argv) > 1 else os.environ.get('HV_LIB_PATH', 'libhvs.so')}: "
      f"median {ts[2]:.3f} ms/step min {ts[0]:.3f} ({16 / ts[2] * 1e3:.1f} img/s)", flush=True)
