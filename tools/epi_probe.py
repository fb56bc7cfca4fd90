"""Is a GEMM epilogue/store-bound?  Time M x N x K for several K (bf16 out, fp32 out, GELU)."""
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
    return s.elapsed_time(e) / iters * 1e3


for M, N in [(102400, 1024), (25600, 2048), (6416, 1024)]:
    for K in (64, 128, 256, 512, 1024):
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        res = []
        for staged in (0, 1):
            lib.hv_gemm_set_staged_epilogue(staged)
            t_bf = timeit(lambda: ops.gemm(a, b))
            t_f32 = timeit(lambda: ops.gemm(a, b, out_dtype=torch.float32))
            t_gelu = timeit(lambda: ops.gemm(a, b, bias=bias, act="gelu"))
            res.append(f"bf16 {t_bf:6.1f} us ({M * N * 2 / t_bf / 1e6:4.2f} TB/s, {2 * M * N * K / t_bf / 1e6:6.1f} "
                       f"TF/s) fp32 {t_f32:6.1f} gelu {t_gelu:6.1f}")
        lib.hv_gemm_set_staged_epilogue(1)
        print(f"M={M:6d} N={N:5d} K={K:5d}: frag {res[0]} || staged {res[1]}", flush=True)
