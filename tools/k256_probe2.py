"""Small-K GEMM: is the 128x128 LDS-DMA kernel store-bound or latency-bound at K=256?
Output dtype (bf16 vs fp32 = 2x the bytes written) and K (64..1024 at fixed M, N) sweeps, plus
torch.mm (hipBLASLt) beside it.  HIP events.  usage: python tools/k256_probe2.py"""
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


M, N = 25600, 2048
for K in (64, 128, 256, 512, 1024):
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    o16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    lib.hv_gemm_set_smallk(0)
    r16 = timeit(lambda: ops.gemm(x, b))
    lib.hv_gemm_set_smallk(2)
    tns = timeit(lambda: ops.gemm(x, b))
    lib.hv_gemm_set_smallk(3)
    tnk = timeit(lambda: ops.gemm(x, b))
    lib.hv_gemm_set_smallk(1)
    t16 = timeit(lambda: ops.gemm(x, b))
    t32 = timeit(lambda: ops.gemm(x, b, out_dtype=torch.float32))
    tmm = timeit(lambda: torch.mm(x, b.t(), out=o16))
    fl = 2.0 * M * N * K
    print(f"K={K:5d}  ring {r16:7.1f}  sk-no-store {tns:7.1f}  sk-no-kloop {tnk:7.1f}  bf16-out {t16:7.1f} us ({fl / t16 / 1e6:6.1f} TF/s, write {M * N * 2 / t16 / 1e6:5.2f} TB/s)  "
          f"fp32-out {t32:7.1f} us (write {M * N * 4 / t32 / 1e6:5.2f} TB/s)  torch.mm {tmm:7.1f} us", flush=True)
# pure write bandwidth reference: fill of the same output
o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
tf = timeit(lambda: o.fill_(1.0))
print(f"fill bf16 [{M}x{N}] {tf:7.1f} us ({M * N * 2 / tf / 1e6:5.2f} TB/s)")
# row pitch: a power-of-two output pitch (4 KiB rows) vs padded pitches, same GEMM
K = 256
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
b = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
for pad in (0, 64, 128, 512):
    big = torch.empty(M, N + pad, device="cuda", dtype=torch.bfloat16)
    view = big[:, :N]
    lib.hv_gemm_set_smallk(3)
    tnk = timeit(lambda: ops.gemm(x, b, out=view))
    lib.hv_gemm_set_smallk(1)
    t = timeit(lambda: ops.gemm(x, b, out=view))
    lib.hv_gemm_set_smallk(0)
    tr = timeit(lambda: ops.gemm(x, b, out=view))
    lib.hv_gemm_set_smallk(1)
    print(f"K=256 ldc={N + pad:5d}: sk {t:7.1f} us (stores only {tnk:7.1f})  ring {tr:7.1f} us", flush=True)
