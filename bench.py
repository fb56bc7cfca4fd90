#!/usr/bin/env python3
"""HybridVision inference throughput on MI355X (BASELINE.json metric, config B).

Workload: hybrid_vision base (353.8M params, reference architecture, random init), 640x640,
batch 16 per GPU, bf16 activations / fp32 coefficients, 20 Sinkhorn iterations, eval mode.
A "step" is one full forward (backbone, mHC transformer, FPN, YOLO head + decode, final
features) over one synthetic batch already resident in HBM; every parameter-only
quantity (Sinkhorn projections, coefficient folds, BN folds, casts) is recomputed inside
every step exactly as the reference recomputes it per forward.

Multi-GPU: inference shards images with no data-path collective ("replicas", weak scaling):
one process per GPU (torchrun), barrier + synchronize around the timed region, time = max
over ranks, value = images processed by all ranks / that time.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "humanoid-vision-system_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GFLOP_PER_IMG_640 = 698.7          # reference graph, SURVEY §8(d) (FlopCounterMode on the oracle)
BF16_PEAK_TFLOPS = 2500.0          # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
METRIC = "COCO 640×640 images/sec at 1/2/4/8 GPUs; single-image p50 latency"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--eager", dest="graph", action="store_false",
                    help="time host-launched steps instead of HIP-graph replays")
    ap.add_argument("--train", dest="train", action="store_true", default=None,
                    help="also time the training step (config C: base 640, bf16, DDP over RCCL when N>1); "
                         "default: on at N=1, off at N>1")
    ap.add_argument("--no-train", dest="train", action="store_false")
    ap.add_argument("--train-batch", type=int, default=16)
    ap.add_argument("--train-steps", type=int, default=4)
    return ap.parse_args()


class GemmTimer:
    """Wraps ops.gemm/conv2d launches with HIP events on the launching stream to measure the
    dominant kernel (the MFMA GEMM) per launch, plus its work 2*M*N*K."""

    def __init__(self, ops):
        self.ops = ops
        self.recs = []
        self._orig = (ops.gemm, ops.conv2d)

    def __enter__(self):
        ops = self.ops
        g0, c0 = self._orig

        def gemm(a, b, **kw):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = g0(a, b, **kw)
            e.record()
            k = b.shape[1]
            m, n = a.shape[0], b.shape[0]
            self.recs.append((s, e, 2.0 * m * n * k, a.element_size() * (m * k + n * k + m * n)))
            return out

        def conv2d(x, w, k, stride, pad, **kw):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = c0(x, w, k, stride, pad, **kw)
            e.record()
            m = out.shape[0] * out.shape[1] * out.shape[2]
            self.recs.append((s, e, 2.0 * m * w.shape[0] * w.shape[1],
                              x.element_size() * (x.numel() + w.numel() + m * w.shape[0])))
            return out

        ops.gemm, ops.conv2d = gemm, conv2d
        return self

    def __exit__(self, *exc):
        self.ops.gemm, self.ops.conv2d = self._orig
        return False

    def summary(self):
        torch.cuda.synchronize()
        ms = sum(r[0].elapsed_time(r[1]) for r in self.recs)
        fl = sum(r[2] for r in self.recs)
        by = sum(r[3] for r in self.recs)
        n = len(self.recs)
        return n, ms / n, fl / n, fl / (ms * 1e-3) / 1e12, by / n


def cpu_baseline(model_cpu_sd, size, threads):
    """Oracle (CPU restatement of the reference path) on the host cores: a bounded sample."""
    from oracle import hv_oracle as O
    torch.set_num_threads(threads)
    x = torch.randn(1, 3, size, size, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        O.system_forward(model_cpu_sd, x, O.BASE)          # warmup
        t0 = time.perf_counter()
        n = 0
        while n < 3 or (time.perf_counter() - t0 < 10 and n < 8):
            O.system_forward(model_cpu_sd, x, O.BASE)
            n += 1
        dt = time.perf_counter() - t0
    return {"value": round(n / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} single-image {size}x{size} fp32 forwards of the oracle (oracle/hv_oracle.py), "
                      f"same random-init weights, after 1 warmup"}


def train_bench(a, dev, world, rank):
    """Config C: base 640x640 bf16 training step -- train-mode forward, YOLOLoss on
    synthetic COCO targets, backward (Sinkhorn autograd included), bucketed gradient all-reduce
    over RCCL overlapped with the backward when N>1, per-group clipping, AdamW."""
    from hv_amd import HybridVisionSystem
    from hv_amd.targets import synthetic_targets
    from hv_amd.trainer import HVTrainer
    torch.manual_seed(0)
    model = HybridVisionSystem({"image_size": a.size, "precision": a.precision, "verbose": False}).to(dev).train()
    tr = HVTrainer(model)
    B = a.train_batch
    x = torch.randn(B, 3, a.size, a.size, device=dev)
    tg = [t.to(dev) for t in synthetic_targets(B, a.size, seed=1000 + rank)]
    for _ in range(2):
        tr.step(x, tg)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.train_steps):
        loss = tr.step(x, tg)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    out = {"metric": "train images/s (forward + YOLOLoss + backward + all-reduce + clip + AdamW)",
           "value": round(world * B * a.train_steps / el, 3), "unit": "images/s",
           "ms_per_step": round(el / a.train_steps * 1e3, 2), "per_gpu_batch": B, "steps": a.train_steps,
           "workload": f"hybrid_vision base {a.size}x{a.size} training, bf16 activations, fp32 params, "
                       f"{'DDP RCCL' if world > 1 else 'single GPU'}",
           "loss": round(loss["total_loss"].item(), 3),
           "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1),
           "model_tflops_reference_graph": round(2095.9 * world * B * a.train_steps / el / 1e3, 2)}
    del tr, model
    torch.cuda.empty_cache()
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from hv_amd import HybridVisionSystem, ops
    torch.manual_seed(0)
    model = HybridVisionSystem({"image_size": a.size, "precision": a.precision, "verbose": False})
    cpu_sd = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu_sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(dev).eval()
    x = torch.randn(a.batch, 3, a.size, a.size, device=dev, generator=None)

    with torch.no_grad():
        for _ in range(2):
            model(x)
        # eager reference timing (host-launched kernels), reported beside the graph number
        torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(3):
            model(x)
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - te) / 3 * 1e3
        step = model.capture(x).replay if a.graph else (lambda: model(x))
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    # dominant-kernel roofline: the MFMA GEMM family, timed with HIP events in one more step
    with torch.no_grad(), GemmTimer(ops) as gt:
        model(x)
    n_l, avg_ms, avg_flop, gemm_tflops, avg_bytes = gt.summary()
    traffic = None
    tf = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
    if a.size == 640 and a.batch == 16 and a.precision == "bf16" and os.path.exists(tf):
        with open(tf) as f:
            traffic = json.load(f).get("gemm", {}).get("bytes_per_launch")

    lat = None
    if rank == 0 and not a.no_latency:
        # streaming config E: single 640x640 frame, hipGraph-captured forward; the frame is copied
        # into the graph's input buffer inside the timed interval
        lat = {}
        frames = torch.randn(8, 1, 3, a.size, a.size, device=dev)
        for mode in ("recompute", "frozen"):
            model.freeze(mode == "frozen")
            with torch.no_grad():
                runner = model.capture(frames[0])
                ts = []
                for i in range(60):
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    runner(frames[i % 8])
                    torch.cuda.synchronize()
                    if i >= 10:
                        ts.append((time.perf_counter() - t1) * 1e3)
            del runner
            ts.sort()
            lat[mode] = {"p50_ms": round(ts[len(ts) // 2], 3), "p95_ms": round(ts[int(len(ts) * 0.95) - 1], 3),
                         "p99_ms": round(ts[-1], 3)}
        model.freeze(False)
        lat["batch"] = 1
        lat["note"] = ("hipGraph replay; 'recompute' re-runs Sinkhorn + coefficient prep per frame like the "
                       "reference, 'frozen' reuses them until a parameter changes (eval streaming)")

    train = None
    if a.train if a.train is not None else world == 1:
        train = train_bench(a, dev, world, rank)

    imgs = world * a.batch * a.steps
    value = imgs / elapsed
    ms_step = elapsed / a.steps * 1e3
    if rank == 0:
        base = cpu_baseline(cpu_sd, a.size, a.cpu_threads) if cpu_sd is not None else None
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "images/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": a.precision, "data": "synthetic (randn images, random-init weights)",
            "config": {"workload": f"hybrid_vision base {a.size}x{a.size} inference, 20 Sinkhorn iters",
                       "model": "hybrid_vision base (353.8M params)", "global_batch": world * a.batch,
                       "per_gpu_batch": a.batch, "seq_len": None, "parallelism": f"replicas{world}"},
            "roofline": {"bound": "mfma", "kernel": "gemm_kernel (bf16 MFMA GEMM / implicit-GEMM conv)",
                         "achieved": round(gemm_tflops, 2), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(gemm_tflops / BF16_PEAK_TFLOPS, 4),
                         "traffic": round(traffic) if traffic else None,
                         "traffic_source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this workload "
                                           "(FETCH x2 gfx950 correction), profiles/r01/pmc_traffic.json",
                         "algorithmic_bytes_per_launch": round(avg_bytes),
                         "launches_per_step": n_l, "avg_launch_ms": round(avg_ms, 4),
                         "avg_flop_per_launch": avg_flop},
            "model_tflops_reference_graph": round(GFLOP_PER_IMG_640 * value / 1e3, 2) if a.size == 640 else None,
            "step_mode": "hipGraph replay of the full forward (Sinkhorn + coefficient prep recomputed every step)"
                         if a.graph else "eager",
            "eager_ms_per_step": round(eager_ms, 3),
            "latency": lat,
            "training": train,
            "cpu_baseline": base,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
