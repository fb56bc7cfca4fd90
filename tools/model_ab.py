"""In-model A/B of a GEMM knob: base 640 bf16 B=16 forward as a hipGraph captured under each
setting (kernel choice is fixed at capture), replays timed in interleaved rounds.

usage: python tools/model_ab.py <knob> <v0> <v1> [batch]
  knob: deep | staged | big | small | train128 | ktail (hv_gemm_set_*),
        mhc (hv_mhc_fused_set_variant), wide (hv_mhc_fused_enable_wide)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem, _lib  # noqa: E402

lib = _lib.lib()
knob, v0, v1 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
B = int(sys.argv[4]) if len(sys.argv) > 4 else 16
setter = {"deep": lib.hv_gemm_set_deep_ring, "staged": lib.hv_gemm_set_staged_epilogue,
          "big": lib.hv_gemm_set_big_tile, "small": lib.hv_gemm_set_small_tile,
          "train128": lib.hv_gemm_set_train128, "ktail": lib.hv_gemm_set_conv_ktail,
          "mhc": lib.hv_mhc_fused_set_variant, "wide": lib.hv_mhc_fused_enable_wide}[knob]
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).cuda().eval()
x = torch.randn(B, 3, 640, 640, device="cuda")
runners = {}
with torch.no_grad():
    m(x)
    for v in (v0, v1):
        setter(v)
        runners[v] = m.capture(x)
    setter(v0)
    res = {v0: [], v1: []}
    for rnd in range(5):
        for v in (v0, v1):
            r = runners[v]
            for _ in range(2):
                r.replay()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(10):
                r.replay()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t) / 10 * 1e3)
for v in (v0, v1):
    ts = sorted(res[v])
    print(f"{knob}={v}: median {ts[len(ts) // 2]:.3f} ms/step  min {ts[0]:.3f}  ({B / ts[len(ts) // 2] * 1e3:.1f} img/s)")
