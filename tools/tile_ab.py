"""A/B of the 64x64 small-grid tile rule on the ViT/head mHC GEMM shapes (HIP events)."""
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
    return s.elapsed_time(e) / iters


for M, N, K in [(6416, 256, 768), (6416, 1024, 256), (6416, 512, 1024), (6416, 256, 1024), (6400, 256, 2304),
                (1600, 512, 1024), (6400, 1024, 512), (25600, 256, 1280)]:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    r = {}
    for mode in (0, 1):
        lib.hv_gemm_set_small_tile(mode)
        r[mode] = (timeit(lambda: ops.gemm(a, b)), ops.gemm(a, b))
    lib.hv_gemm_set_small_tile(1)
    fl = 2.0 * M * N * K
    same = torch.equal(r[0][1], r[1][1])
    print(f"M={M:6d} N={N:5d} K={K:5d}: 64x128 {fl / r[0][0] / 1e9:7.1f} TF/s | 64x64 {fl / r[1][0] / 1e9:7.1f} TF/s"
          f"  bitwise-equal {same}", flush=True)
