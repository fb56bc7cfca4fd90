"""In-model A/B of execution options: base 640 bf16 forward as a hipGraph captured under each
option set (runtime.HVOptions: kernel variants are per call and fixed at capture), replays timed
in interleaved rounds.

usage: python tools/model_ab.py <spec0> <spec1> [batch]
  spec: comma-separated HVOptions fields, e.g. "gemm_variant=16" (HV_GV_NO_BIG),
        "mhc_variant=2", "use_fused_mhc=0,group_qkv=0", or "default"
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd.runtime import HVOptions  # noqa: E402


def parse(spec: str) -> HVOptions:
    kw = {}
    if spec != "default":
        for item in spec.split(","):
            k, v = item.split("=")
            kw[k] = int(v, 0)
    return HVOptions(**kw)


specs = sys.argv[1:3]
B = int(sys.argv[3]) if len(sys.argv) > 3 else 16
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).cuda().eval()
x = torch.randn(B, 3, 640, 640, device="cuda")
runners = {}
with torch.no_grad():
    m(x)
    for sp in specs:
        m.set_options(parse(sp))
        runners[sp] = m.capture(x)
    res = {sp: [] for sp in specs}
    for rnd in range(5):
        for sp in specs:
            r = runners[sp]
            for _ in range(2):
                r.graph.replay()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(10):
                r.graph.replay()
            torch.cuda.synchronize()
            res[sp].append((time.perf_counter() - t) / 10 * 1e3)
for sp in specs:
    ts = sorted(res[sp])
    print(f"{sp}: median {ts[len(ts) // 2]:.3f} ms/step  min {ts[0]:.3f}  ({B / ts[len(ts) // 2] * 1e3:.1f} img/s)")
