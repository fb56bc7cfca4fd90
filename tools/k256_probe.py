"""Small-K GEMM probe: where the time of the LN-epilogue GEMM1 shapes goes (plain product,
+bias+GELU, +LayerNorm epilogue, hipBLASLt torch.mm for scale), each tile forced.  HIP events.
usage: python tools/k256_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ops, _lib  # noqa: E402

lib = _lib.lib()


def timeit(fn, iters=30, warm=5):
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


SHAPES = [(25600, 2048, 256), (102400, 1024, 256), (6416, 1024, 256), (6400, 4096, 512)]
TILES = {"auto": 0, "128x128": 1, "64x128": 2, "128x64": 3, "64x64": 4}
for M, N, K in SHAPES:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    cs = b.float().sum(1)
    mean, rstd = ops.row_stats(x, 1e-5)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    byts = (M * K + N * K + M * N) * 2
    variants = {
        "plain": lambda: ops.gemm(x, b),
        "bias+gelu": lambda: ops.gemm(x, b, bias=bias, act="gelu"),
        "ln+gelu": lambda: ops.gemm(x, b, bias=bias, act="gelu", a_mean=mean, a_rstd=rstd, b_colsum=cs),
    }
    t_mm = timeit(lambda: torch.mm(x, b.t(), out=out))
    print(f"M={M} N={N} K={K}: torch.mm {t_mm:7.1f} us ({fl / t_mm / 1e6:6.1f} TF/s, {byts / t_mm / 1e6:5.2f} TB/s)",
          flush=True)
    for vn, fn in variants.items():
        row = []
        for tn, code in TILES.items():
            lib.hv_gemm_set_force_tile(code)
            try:
                row.append((tn, timeit(fn)))
            except RuntimeError:
                row.append((tn, float("nan")))
        lib.hv_gemm_set_force_tile(0)
        print(f"  {vn:10s} " + "  ".join(f"{tn} {t:7.1f}" for tn, t in row)
              + f"   best {fl / min(t for _, t in row) / 1e6:6.1f} TF/s", flush=True)
