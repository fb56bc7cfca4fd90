"""Per-shape sweep of the LDS-DMA GEMM tiles (per-call variant HV_GV_TILE_MASK) on the bench's weak GEMM
shapes, with their real epilogues (LN-after-product + GELU, K-concat, conv).  HIP events, us.
usage: python tools/tile_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ops  # noqa: E402
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
    return s.elapsed_time(e) / iters * 1e3


def case_ln(M, N, K):
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16) * 0.05
    bias = torch.randn(N, device="cuda")
    cs = b.float().sum(1)
    mean, rstd = ops.row_stats(x, 1e-5)
    return lambda: ops.gemm(x, b, bias=bias, act="gelu", a_mean=mean, a_rstd=rstd, b_colsum=cs), 2.0 * M * N * K


def case_plain(M, N, K, act="gelu"):
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16) * 0.05
    bias = torch.randn(N, device="cuda")
    return lambda: ops.gemm(a, b, bias=bias, act=act), 2.0 * M * N * K


def case_cat(M, N, K1, K2):
    a = torch.randn(M, K1, device="cuda").to(torch.bfloat16)
    a2 = torch.randn(M, K2, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K1 + K2, device="cuda").to(torch.bfloat16) * 0.05
    return lambda: ops.gemm(a, b, a2=a2, out_dtype=torch.float32), 2.0 * M * N * (K1 + K2)


def case_conv(n, h, c, cout, k, s):
    x = torch.randn(n, h, h, c, device="cuda").to(torch.bfloat16)
    w = (torch.randn(cout, k * k * c, device="cuda") * 0.05).to(torch.bfloat16)
    oh = (h + 2 * (k // 2) - k) // s + 1
    return lambda: ops.conv2d(x, w, k, s, k // 2, act="silu"), 2.0 * n * oh * oh * cout * k * k * c


CASES = [
    ("ln 25600x2048x256", lambda: case_ln(25600, 2048, 256)),
    ("ln 102400x1024x256", lambda: case_ln(102400, 1024, 256)),
    ("ln 6416x3072x256", lambda: case_ln(6416, 3072, 256)),
    ("ln 6416x1024x256", lambda: case_ln(6416, 1024, 256)),
    ("ln 6400x4096x512", lambda: case_ln(6400, 4096, 512)),
    ("gemm 6416x512x1024", lambda: case_plain(6416, 512, 1024)),
    ("gemm 25600x1024x2048", lambda: case_plain(25600, 1024, 2048)),
    ("gemm 102400x512x1024", lambda: case_plain(102400, 512, 1024)),
    ("cat 6416x256x(256+512)", lambda: case_cat(6416, 256, 256, 512)),
    ("cat 25600x256x(256+1024)", lambda: case_cat(25600, 256, 256, 1024)),
    ("conv1x1 16x40x256->256", lambda: case_conv(16, 40, 256, 256, 1, 1)),
    ("conv3x3 16x80x256->256", lambda: case_conv(16, 80, 256, 256, 3, 1)),
    ("conv3x3 16x80x256->512", lambda: case_conv(16, 80, 256, 512, 3, 1)),
    ("conv3x3 16x80x512->256", lambda: case_conv(16, 80, 512, 256, 3, 1)),
    ("conv3x3 16x40x512->1024", lambda: case_conv(16, 40, 512, 1024, 3, 1)),
    ("conv3x3 16x40x1024->512", lambda: case_conv(16, 40, 1024, 512, 3, 1)),
    ("conv3x3 16x20x1024->2048", lambda: case_conv(16, 20, 1024, 2048, 3, 1)),
    ("conv3x3 16x20x2048->1024", lambda: case_conv(16, 20, 2048, 1024, 3, 1)),
]
if os.environ.get("HV_SWEEP_ONLY"):
    CASES = [c for c in CASES if os.environ["HV_SWEEP_ONLY"] in c[0]]
print(f"{'case':28s} " + " ".join(f"{n:>9s}" for n in ("auto", "128x128", "64x128", "128x64", "64x64", "256pp", "sk")))
for name, mk in CASES:
    fn, flop = mk()
    row = []
    for code in range(7):
        with use_ctx(RunCtx(dtype=torch.bfloat16, opts=HVOptions(gemm_variant=code))):   # per-call tile
            try:
                row.append(timeit(fn))
            except RuntimeError:
                row.append(float("nan"))
    best = min(v for v in row if v == v)
    print(f"{name:28s} " + " ".join(f"{v:9.1f}" for v in row) + f"   best {flop / best / 1e6:7.1f} TF/s", flush=True)
