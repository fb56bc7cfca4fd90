"""Per-parameter bf16 gradient errors of one training-step group (verdict r5 item 1): the base
model's 224 B=2 bf16 step vs the reference's fp64 gradient norms (fixture train_base_224_b2), beside
the reference's OWN bf16 error (train_base_224_b2_bf16ref).  Prints every parameter of the group
sorted by its share of the group-norm error, and the fp32 HIP step's error for comparison.

    python tools/vit_grad_probe.py [group-prefix, default vit_encoder] > gpurun_out/vit_grad_probe.txt
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "humanoid-vision-system_amd"))

from conftest import GOLDEN, golden  # noqa: E402
from test_gpu_train import _base_train_step  # noqa: E402
from hv_amd.trainer import mhc_group  # noqa: E402


def _patch(mode):
    """Precision bisection: run one part of the ViT in fp32 inside the bf16 step.  Returns the undo."""
    from hv_amd import train_fn as TF
    from hv_amd import train_model as TM
    f32, b16 = torch.float32, torch.bfloat16
    saved = (TF.AttentionFn.apply, TF.linear, TM.attention)

    def undo():
        TF.AttentionFn.apply, TF.linear, TM.attention = saved
    if mode == "attn32":                          # attention core (QK^T, softmax, PV and backward) in fp32
        orig = TF.AttentionFn.apply

        def attn(q, k, v, heads, p, seed):
            if q.dtype != b16:
                return orig(q, k, v, heads, p, seed)
            o = orig(TF.CastFn.apply(q, f32), TF.CastFn.apply(k, f32), TF.CastFn.apply(v, f32), heads, p, seed)
            return TF.CastFn.apply(o, b16)
        TF.AttentionFn.apply = attn
    elif mode == "lin32":                         # the blocks' MLP Linears in fp32
        orig_lin = TF.linear

        def lin(x, l, act="none", p=0.0, out_dtype=None):
            if x.dtype == b16 and out_dtype is None:
                return orig_lin(TF.CastFn.apply(x, f32), l, act, p, out_dtype=b16)
            return orig_lin(x, l, act, p, out_dtype)
        TF.linear = lin
    elif mode == "qkv32":                         # q / k / v / out_proj mHC outputs kept fp32
        orig_att = TM.attention

        def att(a, x, n, H):
            if x.dtype != b16:
                return orig_att(a, x, n, H)
            L = x.shape[0] // n
            q = TM._mhc(a.q_proj, x, H, out_f32=True).view(n, L, -1)
            k = TM._mhc(a.k_proj, x, H, out_f32=True).view(n, L, -1)
            v = TM._mhc(a.v_proj, x, H, out_f32=True).view(n, L, -1)
            p = a.dropout.p
            o = TF.AttentionFn.apply(q, k, v, a.num_heads, p, TF.next_seed() if p > 0 else 0)
            return TM._mhc(a.out_proj, TF.CastFn.apply(o.reshape(n * L, -1), b16), H)
        TM.attention = att
    return undo


def bisect640(modes):
    """Median over the 640 anchor batches (x seeds 7-11) of the ViT groups' bf16-vs-fp32 error, per
    precision variant (bf16 step with one ViT part in fp32)."""
    import numpy as np
    from test_gpu_train import _group_norms
    from oracle import cases
    dev = torch.device("cuda:0")
    res = {m: [] for m in ["base"] + modes}
    for xs in (7,) + tuple(cases.TRAIN640_SEEDS):
        g32 = _group_norms(_base_train_step(dev, "fp32", 2, 640, xs, 11)[2].items())
        for m in res:
            undos = [_patch(part) for part in m.split("+")] if m != "base" else []
            g16 = _group_norms(_base_train_step(dev, "bf16", 2, 640, xs, 11)[2].items())
            for u in reversed(undos):
                u()
            res[m].append({k: abs(g16[k] / v - 1) for k, v in g32.items() if k.startswith("vit")})
            print(f"seed {xs} {m}: {({k: round(v, 4) for k, v in res[m][-1].items()})}", flush=True)
    for m, rs in res.items():
        print(f"MEDIAN {m}: {({k: round(float(np.median([r[k] for r in rs])), 4) for k in rs[0]})}", flush=True)


def stream_ab():
    """640 B=2 bf16-vs-fp32 gradient-group errors (x seeds 7, 8, 9; targets 11), with and without
    the fp32 ViT residual stream (train_model.VIT_F32_STREAM)."""
    from hv_amd import train_model as TM
    from test_gpu_train import _group_norms
    dev = torch.device("cuda:0")
    for xs in (7, 8, 9):
        _, _, n32, _ = _base_train_step(dev, "fp32", 2, 640, xs, 11)
        g32 = _group_norms(n32.items())
        for on in (True, False):
            TM.VIT_F32_STREAM = on
            _, _, n16, _ = _base_train_step(dev, "bf16", 2, 640, xs, 11)
            g16 = _group_norms(n16.items())
            e = {k: round(abs(g16[k] / v - 1), 4) for k, v in g32.items() if k.startswith("vit")}
            print(f"seed {xs} f32_stream={on}: {e}", flush=True)
    TM.VIT_F32_STREAM = True


def determinism():
    """The same 640 B=2 steps twice in one process: are the gradient norms bitwise repeatable?"""
    dev = torch.device("cuda:0")
    for prec in ("fp32", "bf16"):
        a = _base_train_step(dev, prec, 2, 640, 7, 11)[2]
        b = _base_train_step(dev, prec, 2, 640, 7, 11)[2]
        diff = [n for n in a if a[n] != b[n]]
        print(f"{prec}: {len(diff)} of {len(a)} parameter gradient norms differ between two runs; e.g. "
              f"{[(n, a[n], b[n]) for n in diff[:3]]}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "stream_ab":
        return stream_ab()
    if len(sys.argv) > 1 and sys.argv[1] == "determinism":
        return determinism()
    if len(sys.argv) > 1 and sys.argv[1] == "bisect640":
        return bisect640(sys.argv[2:])
    prefix = sys.argv[1] if len(sys.argv) > 1 else "vit_encoder"
    for mode in sys.argv[2:]:
        _patch(mode)
        print(f"patched: {mode}")
    dev = torch.device("cuda:0")
    g = golden("train_base_224_b2")
    gb = golden("train_base_224_b2_bf16ref")
    names = json.load(open(os.path.join(GOLDEN, "train_base_param_names.json")))
    ref64 = {n: float(v) for n, v in zip(names, g["grad_norm_f64"]) if v >= 0}
    refb = {n: float(v) for n, v in zip(names, gb["grad_norm"]) if v >= 0}
    B, S = int(g["B"]), int(g["S"])
    runs = {}
    for prec in ("bf16", "fp32"):
        _, _, norms, fin = _base_train_step(dev, prec, B, S, 1, int(g["target_seed"]))
        runs[prec] = norms
        print(f"{prec}: finite={fin}")
    rows = []
    for n in names:
        if not n.startswith(prefix) or n not in ref64:
            continue
        grp = "mhc" if mhc_group(n) == 0 else "other"
        r = ref64[n]
        rows.append((grp, n, r, runs["bf16"].get(n, 0.0), runs["fp32"].get(n, 0.0), refb.get(n, 0.0)))
    for grp in ("other", "mhc"):
        sel = [x for x in rows if x[0] == grp]
        G = np.sqrt(sum(x[2] ** 2 for x in sel))
        Gh = np.sqrt(sum(x[3] ** 2 for x in sel))
        Gb = np.sqrt(sum(x[5] ** 2 for x in sel))
        print(f"\n== {prefix}/{grp}: group norm f64 {G:.6g}  hip-bf16 {Gh:.6g} (rel {abs(Gh / G - 1):.4f})  "
              f"ref-bf16 {Gb:.6g} (rel {abs(Gb / G - 1):.4f})")
        # share of the squared-norm difference each parameter carries
        tot = sum(abs(x[3] ** 2 - x[2] ** 2) for x in sel) or 1.0
        sel.sort(key=lambda x: -abs(x[3] ** 2 - x[2] ** 2))
        print(f"{'param':60s} {'norm_f64':>11s} {'hip16_rel':>10s} {'hip32_rel':>10s} {'ref16_rel':>10s} {'share':>7s}")
        for _, n, r, h, h32, rb in sel[:40]:
            print(f"{n:60s} {r:11.4e} {h / r - 1 if r else 0:10.4f} {h32 / r - 1 if r else 0:10.4f} "
                  f"{rb / r - 1 if r else 0:10.4f} {abs(h ** 2 - r ** 2) / tot:7.3f}")


if __name__ == "__main__":
    main()
