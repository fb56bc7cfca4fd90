"""256x256 LDS-DMA GEMM kernel: correctness vs torch and timing vs the 128-tile path."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ops, _lib  # noqa: E402

lib = _lib.lib()


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


torch.manual_seed(0)
for M, N, K in [(8192, 8192, 8192), (4096, 4096, 4096), (25600, 1024, 2048), (6400, 2048, 4096), (102400, 512, 1024),
                (25600, 2048, 512), (102400, 1024, 256), (6416, 512, 1024), (1000, 300, 128)]:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    res = {}
    for mode in (0, 2):
        lib.hv_gemm_set_big_tile(mode)
        out = ops.gemm(a, b, bias=bias, act="gelu")
        ms = timeit(lambda: ops.gemm(a, b, bias=bias, act="gelu"), iters=10)
        res[mode] = (out, ms)
    lib.hv_gemm_set_big_tile(1)
    ref = torch.nn.functional.gelu(a.float() @ b.float().t() + bias)
    err = ((res[2][0].float() - ref).norm() / ref.norm()).item()
    err0 = ((res[0][0].float() - ref).norm() / ref.norm()).item()
    fl = 2.0 * M * N * K
    print(f"M={M:6d} N={N:5d} K={K:5d}  128-path {res[0][1]:7.3f} ms {fl / res[0][1] / 1e9:7.1f} TF/s (err {err0:.1e})"
          f" | 256 {res[2][1]:7.3f} ms {fl / res[2][1] / 1e9:7.1f} TF/s (err {err:.1e})", flush=True)
# conv through the 256 kernel
for (n, hw, cin, cout) in [(16, 80, 256, 512), (16, 40, 1024, 512), (16, 20, 2048, 1024)]:
    x = torch.randn(n, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = (torch.randn(cout, 9 * cin, device="cuda") / (9 * cin) ** 0.5).to(torch.bfloat16)
    outs = {}
    for mode in (0, 2):
        lib.hv_gemm_set_big_tile(mode)
        outs[mode] = (ops.conv2d(x, w, 3, 1, 1), timeit(lambda: ops.conv2d(x, w, 3, 1, 1), iters=10))
    lib.hv_gemm_set_big_tile(1)
    d = ((outs[2][0].float() - outs[0][0].float()).norm() / outs[0][0].float().norm()).item()
    fl = 2.0 * n * hw * hw * cout * 9 * cin
    print(f"conv {hw} {cin}->{cout}: 128 {fl / outs[0][1] / 1e9:7.1f} TF/s | 256 {fl / outs[2][1] / 1e9:7.1f} TF/s "
          f"(rel diff {d:.1e})", flush=True)
