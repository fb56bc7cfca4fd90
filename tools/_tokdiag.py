import os, sys
sys.path[:0] = ["/root/repo", "/root/repo/humanoid-vision-system_amd"]
import torch
from hv_amd import ManifoldHyperConnection, _lib, ops
def timed(fn, n=10):
    fn(); s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / n
for T in (401, 1604, 4010):
    ms = [ManifoldHyperConnection(256, expansion_rate=2).cuda().eval() for _ in range(3)]
    ps = [m.plan() for m in ms]
    x = torch.randn(T, 256, device="cuda").to(torch.bfloat16)
    for n in (1, 3):
        for tag, v in (("pf2", 0), ("pf3", 31), ("pf4", 32), ("nt", 33), ("coal", 34), ("coal_pf4", 35)):
            vv = _lib.MV_TOK | _lib.MV_TOK16 | v
            t = min(timed(lambda: ops.mhc_fused_group(x, ps[:n], vv)) for _ in range(3))
            wg = -(-T // 16) * n
            print(f"T={T:5d} n={n} {tag:8s}: {t*1e3:7.1f} us  ({wg} WGs, {2.0*1.97e6*wg/ (t*1e-3) / 1e9 / min(wg,256):.1f} GB/s per busy CU)", flush=True)
