"""Training-step diagnostics on the GPU: bf16-vs-fp32 per-parameter gradient agreement on
the tiny config, and the base-config training step time (forward + YOLOLoss + backward +
clip + AdamW) at a few batch sizes.

usage: python tools/train_diag.py [grads|time|all] [batch] [size] [train128 0|1]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd.targets import synthetic_targets  # noqa: E402
from hv_amd.trainer import HVTrainer  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "all"
dev = torch.device("cuda")
if os.environ.get("HV_GEMM_VARIANT"):
    # A/B only: the training forward / backward run outside any RunCtx (the autograd engine's
    # device thread would not see a context), so the process-wide default options are patched here
    from hv_amd import runtime as _rt
    _rt.DEFAULT_OPTIONS = _rt.HVOptions(gemm_variant=int(os.environ["HV_GEMM_VARIANT"], 0))


def tiny(prec):
    from oracle import weights as W
    m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False, precision=prec))
    W.load_formula_weights(m, "wc")
    m = m.to(dev).train()
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    return m


if what in ("grads", "all"):
    B, S = 2, 64
    x = torch.randn(B, 3, S, S, device=dev)
    tg = [t.to(dev) for t in synthetic_targets(B, S, seed=3)]
    res = {}
    for prec in ("fp32", "bf16"):
        m = tiny(prec)
        l = m(x, targets=tg, compute_loss=True)["loss"]["total_loss"]
        l.backward()
        res[prec] = ({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}, l.item())
    print("loss fp32", res["fp32"][1], "bf16", res["bf16"][1])
    rows = []
    for n, g in res["fp32"][0].items():
        h = res["bf16"][0][n]
        rows.append(((h - g).norm().item() / (g.norm().item() + 1e-30), g.norm().item(), n))
    rows.sort(reverse=True)
    for r in rows[:25]:
        print(f"{r[0]:10.3e} |g|={r[1]:10.3e} {r[2]}")
    tot32 = torch.cat([g.flatten() for g in res["fp32"][0].values()])
    tot16 = torch.cat([res["bf16"][0][n].flatten() for n in res["fp32"][0]])
    print("concat rel", ((tot16 - tot32).norm() / tot32.norm()).item())
    print("median rel", sorted(r[0] for r in rows)[len(rows) // 2])

if what in ("time", "all"):
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 640
    torch.manual_seed(0)
    m = HybridVisionSystem({"image_size": S, "precision": "bf16", "verbose": False}).to(dev).train()
    tr = HVTrainer(m, monitor_every=0)   # metrics-only monitor off while timing kernels
    x = torch.randn(B, 3, S, S, device=dev)
    tg = [t.to(dev) for t in synthetic_targets(B, S, seed=3)]
    for i in range(2):
        tr.step(x, tg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 3
    for i in range(n):
        loss = tr.step(x, tg)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    # host-side cost of one step (launch + autograd bookkeeping) with the GPU kept busy
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    tr.step(x, tg)
    host_ms = (time.perf_counter() - h0) * 1e3
    torch.cuda.synchronize()
    print(f"host time of one step (no sync inside) {host_ms:.1f} ms")
    print(f"train step B={B} S={S}: {dt * 1e3:.1f} ms  {B / dt:.2f} img/s  loss={loss['total_loss'].item():.3f}"
          f"  mem={torch.cuda.max_memory_allocated() / 2**30:.1f} GiB")
