"""Latency structure of the small-grid GEMMs of the B=1 frame (401-token ViT, 20x20 head):
per-launch time inside a captured hipGraph of 50 launches, over K and N, per tile variant.

usage: python tools/small_gemm_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ops  # noqa: E402
from hv_amd import _lib as L  # noqa: E402


def per_launch_us(fn, n=50):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (5 * n)


def main():
    variants = {"auto": 0, "no_deep8": L.GV_NO_DEEP8, "t64x64_d8": L.GV_TILE_64x64 | L.GV_DEEP8,
                "t64x64_d4": L.GV_TILE_64x64 | L.GV_NO_DEEP8, "shallow": L.GV_SHALLOW}
    print(f"{'M':>6}{'N':>6}{'K':>6}  " + "  ".join(f"{k:>10}" for k in variants))
    for M in (401, 1600):
        for N in (256, 768, 1024):
            for K in (64, 256, 512, 768, 1024):
                a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
                b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
                row = []
                for name, v in variants.items():
                    if v is None:
                        row.append("       n/a")
                        continue
                    us = per_launch_us(lambda: ops.gemm(a, b, variant=v) if v else ops.gemm(a, b))
                    row.append(f"{us:10.2f}")
                print(f"{M:>6}{N:>6}{K:>6}  " + "  ".join(row), flush=True)
    # empty-kernel floor: a 1x1 GEMM tile
    a = torch.randn(16, 64, device="cuda").to(torch.bfloat16)
    b = torch.randn(16, 64, device="cuda").to(torch.bfloat16)
    print(f"floor (16x16x64): {per_launch_us(lambda: ops.gemm(a, b)):.2f} us")
    x = torch.randn(401, 256, device="cuda").to(torch.bfloat16)
    print(f"copy 401x256 bf16 (torch): {per_launch_us(lambda: x.clone()):.2f} us")


if __name__ == "__main__":
    with torch.no_grad():
        main()
