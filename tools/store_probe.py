"""Output-stream probe for the small-K LN GEMM (25600 x 2048 x 256): does the output row stride
(power-of-two 4 KiB vs padded) change the store-bound time?  HIP events, us."""
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


for M, N, K in [(25600, 2048, 256), (102400, 1024, 256), (6416, 3072, 256)]:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    mean, rstd = ops.row_stats(x, 1e-5)
    cs = b.float().sum(1)
    row = []
    for pad in (0, 8, 64, 128, 256):
        buf = torch.empty(M, N + pad, device="cuda", dtype=torch.bfloat16)
        out = buf[:, :N]
        for v in (_lib.GV_TILE_SMALLK, _lib.GV_TILE_128x128):
            t = timeit(lambda: ops.gemm(x, b, bias=bias, act="gelu", a_mean=mean, a_rstd=rstd, b_colsum=cs,
                                         out=out, variant=v))
            row.append(f"pad{pad}/{'sk' if v == _lib.GV_TILE_SMALLK else 'ring'} {t:7.1f}")
    # a pure store-stream reference: a copy of the same output bytes
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    z = torch.empty_like(y)
    row.append(f"copy {timeit(lambda: z.copy_(y)):7.1f}")
    print(f"{M}x{N}x{K}: " + "  ".join(row), flush=True)
