"""Sinkhorn group micro-benchmark: the model's matrix sets timed alone (graph replay of one
grouped forward).  usage: python tools/sk_bench.py  (run under rocprofv3 --kernel-trace --stats
for the per-kernel split)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ops  # noqa: E402

# the base model's Sinkhorn matrices (D: count), 20 iterations each
MODEL = {32: 3, 64: 6, 128: 9, 256: 50, 512: 6, 1024: 1, 1792: 1}
SETS = {
    "d1792": {1792: 1},
    "d1024": {1024: 1},
    "d512x6": {512: 6},
    "large": {512: 6, 1024: 1, 1792: 1},
    "small": {32: 3, 64: 6, 128: 9, 256: 50},
    "model": MODEL,
}


def main():
    dev = torch.device("cuda:0")
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(SETS)
    for name in names:
        raws = [torch.randn(d, d, device=dev) for d, c in SETS[name].items() for _ in range(c)]
        g = ops.SinkhornGroup(raws, [20] * len(raws), dev)
        g.run()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                g.run()
        torch.cuda.synchronize()
        for _ in range(5):
            graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            graph.replay()
        torch.cuda.synchronize()
        print(f"{name:8s} {(time.perf_counter() - t0) / 50 * 1e6:8.1f} us per grouped forward", flush=True)


if __name__ == "__main__":
    main()
