"""HBM ceiling probe on this box: torch's vectorised fill (write only) and copy (read + write) of
1-2 GiB buffers, HIP events, best of 10 -- the practical stream rates the write-bound kernels
(small-K GEMM epilogues, training epilogues, decode) are compared against."""
import torch

dev = torch.device("cuda")
a = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
b = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
c = torch.empty(1 << 30, dtype=torch.uint8, device=dev)


def best(fn, nbytes, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    t = min(ts)
    return nbytes / (t * 1e-3) / 1e12, t


w, tw = best(lambda: a.fill_(1), a.numel())
rw, trw = best(lambda: c.copy_(b), 2 * b.numel())
print(f"write (fill 2 GiB): {w:.2f} TB/s ({tw:.3f} ms); read+write (copy 1 GiB): {rw:.2f} TB/s ({trw:.3f} ms)")
