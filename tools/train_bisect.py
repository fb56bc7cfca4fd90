"""Determinism probe of the training step: two eager HVTrainers (and one graph trainer) on the same
batches, tiny config, dropout off -- prints per-step losses and whether the parameters stay
bitwise equal.  usage: python tools/train_bisect.py [gemm_variant] [precision]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem, runtime  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402
from oracle import weights as W  # noqa: E402

v = int(sys.argv[1], 0) if len(sys.argv) > 1 else 0
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
me = int(sys.argv[3]) if len(sys.argv) > 3 else 4          # monitor_every of all three trainers
runtime.DEFAULT_OPTIONS = runtime.HVOptions(gemm_variant=v)
dev = torch.device("cuda")


def tiny():
    m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False, precision=prec))
    W.load_formula_weights(m, "wc")
    m = m.to(dev).train()
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    return m


ms = [tiny(), tiny(), tiny()]
trs = [HVTrainer(ms[0], lr=1e-3, monitor_every=me), HVTrainer(ms[1], lr=1e-3, monitor_every=me),
       HVTrainer(ms[2], lr=1e-3, monitor_every=me, graph=True)]
gen = torch.Generator().manual_seed(5)
B, S = 2, 96
for step in range(4):
    x = torch.randn(B, 3, S, S, generator=gen).to(dev)
    tg = [t.to(dev) for t in synthetic_targets(B, S, seed=20 + step)]
    ls = [float(t.step(x, tg)["total_loss"]) for t in trs]
    torch.cuda.synchronize()
    same = []
    for j in (1, 2):
        bad = [n for (n, pa), (_, pb) in zip(ms[0].named_parameters(), ms[j].named_parameters())
               if not torch.equal(pa, pb)]
        same.append(f"{len(bad)} differ" + (f" (first {bad[0]})" if bad else ""))
    print(f"variant {v:#x} {prec} monitor_every {me} step {step}: eager {ls[0]:.4f} eager2 {ls[1]:.4f} graph {ls[2]:.4f} | "
          f"eager2: {same[0]} | graph: {same[1]}", flush=True)
    pe, pg = trs[0].last_predictions, trs[2].last_predictions
    diffs = {k: float((pe[k].float() - pg[k].float()).abs().max()) for k in pe}
    hist = [n for (n, ba), (_, bb) in zip(ms[0].named_buffers(), ms[2].named_buffers())
            if "convergence_history" in n and not torch.equal(ba, bb)]
    print(f"   predictions max|eager - graph| {diffs}; Sinkhorn histories differing: {len(hist)}", flush=True)
