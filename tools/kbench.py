"""Kernel microbenchmarks (HIP events): fused mHC sites and representative GEMM/conv shapes.

usage: python tools/kbench.py [what...]   what in {mhc, gemm, all}
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ManifoldHyperConnection, ops  # noqa: E402
from hv_amd import manifold as MF  # noqa: E402
from hv_amd.runtime import HVOptions, RunCtx, use_ctx  # noqa: E402


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


def mhc_bench():
    for D, e, T in [(32, 4, 1638400), (64, 4, 1638400), (64, 4, 409600), (128, 4, 102400), (256, 4, 25600),
                    (256, 2, 6416), (256, 2, 102400), (512, 4, 6400)]:
        m = ManifoldHyperConnection(D, expansion_rate=e).cuda().eval()
        x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
        p = m.plan()
        Hd = D * e
        fl = 2.0 * T * (D * 2 * Hd + 2 * Hd * Hd + (D + Hd) * D)
        for fused in (True, False):
            if fused and not ops.mhc_fused_supported(D, Hd, torch.bfloat16):
                continue
            with use_ctx(RunCtx(dtype=torch.bfloat16, opts=HVOptions(use_fused_mhc=fused))):
                ms = timeit(lambda: MF.mhc_apply(x, p))
            print(f"mhc D={D:4d} Hd={Hd:4d} T={T:8d} {'fused  ' if fused else 'unfused'} {ms:8.3f} ms "
                  f"{fl / ms / 1e9:8.1f} TF/s (executed)")


def gemm_bench():
    for M, N, K in [(102400, 512, 1024), (25600, 1024, 2048), (6400, 2048, 4096), (8192, 8192, 8192),
                    (1638400, 128, 256), (102400, 1024, 128)]:
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        ms = timeit(lambda: ops.gemm(a, b), iters=10)
        print(f"gemm M={M:8d} N={N:5d} K={K:5d} {ms:8.3f} ms {2.0 * M * N * K / ms / 1e9:8.1f} TF/s")
    for (n, hw, cin, cout) in [(16, 80, 256, 512), (16, 40, 1024, 512), (16, 20, 2048, 1024), (16, 320, 32, 64)]:
        x = torch.randn(n, hw, hw, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(cout, 9 * cin, device="cuda").to(torch.bfloat16)
        ms = timeit(lambda: ops.conv2d(x, w, 3, 1, 1), iters=10)
        print(f"conv3x3 n={n} hw={hw} {cin}->{cout} {ms:8.3f} ms {2.0 * n * hw * hw * cout * 9 * cin / ms / 1e9:8.1f} TF/s")


if __name__ == "__main__":
    what = sys.argv[1:] or ["all"]
    with torch.no_grad():
        if "mhc" in what or "all" in what:
            mhc_bench()
        if "gemm" in what or "all" in what:
            gemm_bench()
