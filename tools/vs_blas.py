"""Our LDS-DMA GEMM vs torch.mm (hipBLASLt) on the model's GEMM shapes (bf16, HIP events).
Cold-weight effects are excluded on both sides (same operands looped)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ops  # noqa: E402


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
    return s.elapsed_time(e) / iters


shapes = [(25600, 1024, 2048), (6416, 512, 1024), (25600, 2048, 256), (6416, 1024, 256), (6400, 2048, 4096),
          (6416, 256, 768), (102400, 512, 1024), (102400, 1024, 256), (6400, 4096, 512), (8192, 8192, 8192)]
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    fl = 2.0 * M * N * K
    t_ours = timeit(lambda: ops.gemm(a, b))
    bt = b.t()
    t_blas = timeit(lambda: torch.mm(a, bt))
    print(f"M={M:6d} N={N:5d} K={K:5d}: ours {fl / t_ours / 1e9:7.1f} TF/s  torch.mm {fl / t_blas / 1e9:7.1f} TF/s",
          flush=True)
