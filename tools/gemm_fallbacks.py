"""Which training-step GEMMs leave the LDS-DMA family: one eager base-640 training step with
hv_gemm wrapped to log every call whose descriptor fails the LDS-DMA kernel's shape rules
(K % 64, lda / ldb % 8, A2 k1 % 64, LN prologue without b_colsum).
usage: python tools/gemm_fallbacks.py [batch]"""
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem, _lib as L  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
lib = L.lib()
orig = lib.hv_gemm
seen = Counter()


def wrapped(dp, stream):
    d = dp._obj
    bad = []
    if d.conv_k == 0 and d.K % 64:
        bad.append("K%64")
    if d.conv_k > 0 and d.K % 64:
        bad.append("convK%64")
    if d.a_mean and (not d.b_colsum or d.A2 or d.conv_k > 0):
        bad.append("LN")
    if d.A2 and d.k1 % 64:
        bad.append("k1%64")
    if d.conv_transposed:
        bad.append("convT")
    if bad:
        seen[(tuple(bad), d.M, d.N, d.K, d.conv_k, d.conv_c, d.epi_mode, d.dtype)] += 1
    return orig(dp, stream)


lib.hv_gemm = wrapped
dev = torch.device("cuda")
x = torch.randn(B, 3, 640, 640, device=dev)
tg = [t.to(dev) for t in synthetic_targets(B, 640, seed=3)]
torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "precision": "bf16", "verbose": False}).to(dev).train()
tr = HVTrainer(m, monitor_every=0, graph=False)
tr.step(x, tg)
seen.clear()
tr.step(x, tg)
torch.cuda.synchronize()
print("reason, M, N, K, conv_k, conv_c, epi_mode, dtype : calls per step")
for k, v in sorted(seen.items(), key=lambda kv: -kv[0][1] * kv[0][2]):
    print(k, v)
