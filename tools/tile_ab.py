"""A/B of GEMM tile rules (HIP events): `small` = 64x64 small-grid tiles on/off; `big` = the
256x256 ping-pong kernel off / forced; `deep` = 2-buffer vs deeper LDS-DMA rings."""
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


which = sys.argv[1] if len(sys.argv) > 1 else "small"
setter = {"small": lib.hv_gemm_set_small_tile, "big": lib.hv_gemm_set_big_tile,
          "deep": lib.hv_gemm_set_deep_ring}[which]
modes = (0, 2) if which == "big" else (0, 1)
default = 1
shapes = ([(6416, 256, 768), (6416, 1024, 256), (6416, 512, 1024), (6416, 256, 1024), (6400, 256, 2304),
           (1600, 512, 1024), (6400, 1024, 512), (25600, 256, 1280)] if which in ("small", "deep") else
          [(25600, 1024, 2048), (6400, 2048, 4096), (102400, 512, 1024), (25600, 2048, 256), (102400, 1024, 256),
           (6400, 4096, 512), (25600, 512, 1536), (8192, 8192, 8192), (4096, 4096, 4096), (1000, 520, 640)])
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    r = {}
    for mode in modes:
        setter(mode)
        r[mode] = (timeit(lambda: ops.gemm(a, b)), ops.gemm(a, b))
    setter(default)
    fl = 2.0 * M * N * K
    same = torch.equal(r[modes[0]][1], r[modes[1]][1])
    print(f"M={M:6d} N={N:5d} K={K:5d}: mode {modes[0]} {fl / r[modes[0]][0] / 1e9:7.1f} TF/s | mode {modes[1]} "
          f"{fl / r[modes[1]][0] / 1e9:7.1f} TF/s  bitwise-equal {same}", flush=True)
