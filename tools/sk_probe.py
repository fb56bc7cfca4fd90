"""Persistent small-K GEMM diagnostics: full kernel vs the DIAG variants (no stores / no k-loop) at
the in-model LN-epilogue shapes, plus the ring tile for comparison.  HIP events, us.
usage: python tools/sk_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import _lib, ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


SK = _lib.GV_TILE_SMALLK
variants = {"sk": SK, "sk_nostore": SK | _lib.GV_SK_DIAG1, "sk_noloop": SK | _lib.GV_SK_DIAG2,
            "ring128": _lib.GV_TILE_128x128, "ring64x128": _lib.GV_TILE_64x128}
extra = os.environ.get("HV_SK_EXTRA")
if extra:
    for kv in extra.split(","):
        k, v = kv.split("=")
        variants[k] = int(v, 0)
print(f"{'shape':24s} " + " ".join(f"{k:>11s}" for k in variants))
for M, N, K, ln in [(25600, 2048, 256, True), (102400, 1024, 256, True), (6416, 3072, 256, True),
                    (6400, 4096, 512, True), (6416, 1024, 256, True), (25600, 256, 256, False),
                    (102400, 256, 256, False), (409600, 64, 64, False)]:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    if ln:
        mean, rstd = ops.row_stats(x, 1e-5)
        cs = b.float().sum(1)
        f = lambda v: ops.gemm(x, b, bias=bias, act="gelu", a_mean=mean, a_rstd=rstd, b_colsum=cs, variant=v)  # noqa
    else:
        f = lambda v: ops.gemm(x, b, bias=bias, act="silu", variant=v)  # noqa: E731
    row = []
    for k, v in variants.items():
        try:
            row.append(f"{timeit(lambda: f(v)):11.1f}")
        except Exception as ex:  # noqa: BLE001
            row.append(f"{'n/a':>11s}")
    print(f"{M}x{N}x{K}{'+ln' if ln else '':4s} ".ljust(25) + " ".join(row), flush=True)
