#!/usr/bin/env python3
"""Golden-vector generator: runs the REFERENCE implementation (read-only import from
/root/reference) with shims S1-S7 and writes small fixtures to
tests/golden/.  TEST INFRASTRUCTURE ONLY -- runs in the build container, never on the
GPU box and never as part of the product.  The reference's source is not copied:
it is imported at run time; only its outputs (inputs + expected outputs) are stored.

Weights come from oracle/weights.py (regenerated from a formula on both sides).

Usage:  python oracle/gen_golden.py [--only sinkhorn,mhc,blocks,model,...,bf16ref] [--bf16ref mhc,model,train]
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REF = os.environ.get("HV_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REF)

from oracle import weights as W  # noqa: E402
from oracle.cases import (MHC_CASES, MHC_LARGE_CASES, MODEL_CASES, SK_CASES, STAB_CASES, gen_seed,  # noqa: E402
                          mhc_input, mhc_input_large, mhc_large_rows, sinkhorn_raw, stab_inputs)

_TINY = {"on": False}


def apply_shims():
    """Monkey-patch the reference classes with S1-S7 and the tiny-config knobs."""
    import src.models.manifold_layers as ml
    import src.models.vision_backbone as vb
    import src.models.vit_encoder_decoder as ve
    import src.models.yolo_head as yh
    import src.models.hybrid_vision as hv

    # S1: 2-D Sinkhorn input goes through the 3-D path (m = matrix.shape[-1]).
    sk_fwd = ml.SinkhornKnoppProjection.forward

    def sk_forward(self, matrix, return_history=False):
        if matrix.dim() == 2:
            r = sk_fwd(self, matrix.unsqueeze(0), return_history)
            if return_history:
                return r[0].squeeze(0), r[1]
            return r.squeeze(0)
        return sk_fwd(self, matrix, return_history)
    ml.SinkhornKnoppProjection.forward = sk_forward

    # S2: a 4-D NCHW map handed to mHC is processed channels-last.
    mhc_fwd = ml.ManifoldHyperConnection.forward

    def mhc_forward(self, x):
        if x.dim() == 4:
            return mhc_fwd(self, x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        return mhc_fwd(self, x)
    ml.ManifoldHyperConnection.forward = mhc_forward

    # tiny config knobs
    mhc_init = ml.ManifoldHyperConnection.__init__

    def mhc_init_w(self, *a, **k):
        if _TINY["on"]:
            k["sk_iterations"] = 5
        mhc_init(self, *a, **k)
    ml.ManifoldHyperConnection.__init__ = mhc_init_w
    bb_init = vb.HybridVisionBackbone.__init__

    def bb_init_w(self, *a, **k):
        if _TINY["on"]:
            k["num_blocks"] = [1, 1, 1, 1]
        bb_init(self, *a, **k)
    vb.HybridVisionBackbone.__init__ = bb_init_w
    hv.HybridVisionBackbone = vb.HybridVisionBackbone
    he_init = ve.HybridVisionEncoder.__init__

    def he_init_w(self, *a, **k):
        if _TINY["on"]:
            k["vit_depth"] = 1
        he_init(self, *a, **k)
    ve.HybridVisionEncoder.__init__ = he_init_w

    # S3: interpolate the 256 learned patch positions to H*W, keeping the CLS slot.
    def pe_forward(self, x):
        B = x.shape[0]
        x = self.projection(x).flatten(2).transpose(1, 2)
        x = self.mhc_enhance(x)
        x = torch.cat([self.cls_token.expand(B, -1, -1), x], dim=1)
        pe = self.position_embeddings
        if pe.shape[1] != x.shape[1]:
            body = F.interpolate(pe[:, 1:].transpose(1, 2), size=(x.shape[1] - 1,),
                                 mode="linear").transpose(1, 2)
            pe = torch.cat([pe[:, :1], body], dim=1)
        return self.norm(x + pe)
    ve.PatchEmbedding.forward = pe_forward

    # S4: per-scale anchors [S, A, 1, 1, 4] (only w, h are used by the decoder).
    def gen_anchors(self):
        rows = []
        for sizes in self.anchor_sizes:
            rows.append(torch.tensor([[0.5, 0.5, w / 416.0, h / 416.0] for (w, h) in sizes]
                                     ).view(len(sizes), 1, 1, 4))
        return torch.stack(rows)
    yh.YOLOAnchorGenerator._generate_anchors = gen_anchors

    # S5: grid view (1,1,H,W,1) -> boxes [B, A, H, W, 4].
    def dec_forward(self, predictions, anchors, grid_size):
        B, A, H, W_, _ = predictions.shape
        xy = torch.sigmoid(predictions[..., 0:2])
        wh = predictions[..., 2:4]
        obj = torch.sigmoid(predictions[..., 4:5])
        cls = torch.sigmoid(predictions[..., 5:])
        gy, gx = torch.meshgrid(torch.arange(H), torch.arange(W_), indexing="ij")
        gx = gx.view(1, 1, H, W_, 1)
        gy = gy.view(1, 1, H, W_, 1)
        bx = (gx + xy[..., 0:1]) / W_
        by = (gy + xy[..., 1:2]) / H
        bw = anchors[..., 2:3] * torch.exp(wh[..., 0:1])
        bh = anchors[..., 3:4] * torch.exp(wh[..., 1:2])
        boxes = torch.cat([bx - bw / 2, by - bh / 2, bx + bw / 2, by + bh / 2], dim=-1)
        scores = obj * cls
        cs, ci = torch.max(scores, dim=-1)
        return {"boxes": boxes, "scores": scores, "class_scores": cs, "class_indices": ci,
                "objectness": obj, "raw_predictions": predictions}
    yh.YOLODecoder.forward = dec_forward

    # S6: the pooled [B, 1792] vector goes through output_projection[2:] only.
    def final_feats(self, fused):
        lst = [F.adaptive_avg_pool2d(fused[k], (1, 1)).flatten(1)
               for k in ("fused_small", "fused_medium", "fused_large") if k in fused]
        c = self.final_fusion(torch.cat(lst, dim=1))
        return self.output_projection[2:](c)
    hv.HybridVisionSystem._extract_final_features = final_feats

    # S7: get_stability_metrics must skip the root module.
    def stab(self):
        out = {}
        for name, m in self.named_modules():
            if m is self or not hasattr(m, "get_stability_metrics"):
                continue
            for k, v in m.get_stability_metrics().items():
                out[f"{name}.{k}"] = v
        return out
    hv.HybridVisionSystem.get_stability_metrics = stab
    return ml, vb, ve, yh, hv


def save(name, **arrs):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrs.items()})
    print(f"  wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


def gen_sinkhorn(ml):
    print("G1 sinkhorn")
    for fam in ("wc", "init"):
        for D, it in SK_CASES:
            raw = sinkhorn_raw(D, it, fam).requires_grad_(True)
            sk = ml.SinkhornKnoppProjection(num_iterations=it)
            M = sk(raw)
            gG = gen_seed(D, it, 3)
            G = torch.randn(D, D, generator=gG)
            (M * G).sum().backward()
            rec = {"D": D, "iters": it, "history": sk.convergence_history.clone(),
                   "row_sums": M.sum(1), "col_sums": M.sum(0)}
            idx = torch.tensor([0, 1, D // 2, D - 1])
            rec["rows"] = M[idx]
            rec["cols"] = M[:, idx].T
            rec["grad_rows"] = raw.grad[idx]
            if D <= 256:
                rec["M"] = M
                rec["grad"] = raw.grad
            save(f"sk_{fam}_D{D}_it{it}", **rec)
    # the reference test's own cases (test_models.py:33-100): batched 3-D inputs
    g = torch.Generator().manual_seed(7)
    mat = torch.randn(4, 8, 8, generator=g)
    sk = ml.SinkhornKnoppProjection(num_iterations=20)
    save("sk_batched_4x8x8", raw=mat, M=sk(mat), history=sk.convergence_history.clone())
    mat = torch.randn(2, 5, 7, generator=g)
    sk = ml.SinkhornKnoppProjection(num_iterations=10)
    save("sk_batched_2x5x7", raw=mat, M=sk(mat), history=sk.convergence_history.clone())


# ------------------------------------------------------------------ G1b stability monitor
def gen_stability(ml):
    """ManifoldHyperConnection._monitor_stability (manifold_layers.py:282-316) of the reference,
    called on the reference's own Sinkhorn output: eigenvalues buffer (fp32 eigvalsh), the
    monitoring_metrics dict and the circular-history entry."""
    print("G1b stability")
    for D, fam in STAB_CASES:
        raw = sinkhorn_raw(D, 20, fam)
        with torch.no_grad():
            H = ml.SinkhornKnoppProjection(num_iterations=20)(raw)
            x_in, x_out = stab_inputs(D, fam)
            m = ml.ManifoldHyperConnection(D, expansion_rate=2)
            m._monitor_stability(H, x_in, x_out)
        mm = m.monitoring_metrics
        rec = {"D": D, "eigenvalues": m.eigenvalues.clone(), "history0": m.signal_ratio_history[0].clone(),
               "signal_ratio": mm["signal_ratio"], "row_sum_error": mm["row_sum_error"],
               "col_sum_error": mm["col_sum_error"], "max_eigenvalue": mm["max_eigenvalue"],
               "min_eigenvalue": mm["min_eigenvalue"]}
        if D <= 256:
            rec["H"] = H
        save(f"stab_{fam}_D{D}", **rec)


# ------------------------------------------------------------------ G2 mHC


def gen_mhc(ml):
    print("G2 mhc")
    for fam in ("wc", "init"):
        for D, e in MHC_CASES:
            torch.manual_seed(0)
            m = ml.ManifoldHyperConnection(D, expansion_rate=e).eval()
            W.load_formula_weights(m, fam)
            x = mhc_input(D, e).requires_grad_(True)
            y = m(x)
            G = torch.randn(64, D, generator=gen_seed(D, e, 12))
            (y * G).sum().backward()
            with torch.no_grad():
                m64 = ml.ManifoldHyperConnection(D, expansion_rate=e).double().eval()
                W.load_formula_weights(m64, fam)
                y64 = m64(x.detach().double())
            ghres = m.H_res_raw.grad if D <= 256 else m.H_res_raw.grad[:4]
            save(f"mhc_{fam}_D{D}_e{e}", x=x, y=y, y64=y64.float(), gx=x.grad,
                 g_hres=ghres, g_hpre_sum=m.H_pre_raw.grad.abs().sum(),
                 g_w1_sum=m.mlp[0].weight.grad.abs().sum())


def gen_mhc_large(ml):
    """mHC at the token counts where the automatic policy selects each large-T kernel
    (cases.MHC_LARGE_CASES): the reference's fp64 forward on a row subsample (the chain is
    per-token), plus the input checksum the test verifies its regenerated x against."""
    print("G2b mhc large-T")
    for fam in ("wc", "init"):
        for D, e, T in MHC_LARGE_CASES:
            x = mhc_input_large(D, e, T)
            rows = mhc_large_rows(T)
            with torch.no_grad():
                m64 = ml.ManifoldHyperConnection(D, expansion_rate=e).double().eval()
                W.load_formula_weights(m64, fam)
                y64 = torch.cat([m64(x[i:i + 8192].double()) for i in range(0, T, 8192)])
            save(f"mhc_{fam}_D{D}_e{e}_T{T}", rows=rows, y64=y64[rows].float(), x_sum=x.double().sum(),
                 x_abs_sum=x.double().abs().sum(), T=T)


# ------------------------------------------------------------------ G3 blocks
def gen_blocks(ml, vb, ve, yh):
    print("G3 blocks")
    fam = "wc"
    # ConvMHCLayer stem.0 config (3->32, s2) and 64->64 (residual path)
    for (cin, cout, k, s, HW) in [(3, 32, 3, 2, 32), (64, 64, 3, 1, 16), (64, 128, 3, 2, 16)]:
        torch.manual_seed(0)
        m = vb.ConvMHCLayer(cin, cout, kernel_size=k, stride=s).eval()
        W.load_formula_weights(m, fam)
        x = torch.randn(2, cin, HW, HW, generator=gen_seed(cin, cout, HW))
        with torch.no_grad():
            save(f"convmhc_{cin}_{cout}_s{s}", x=x, y=m(x))
    torch.manual_seed(0)
    m = vb.ResidualMHCLayer(128, num_blocks=2, expansion_rate=4, bottleneck=True).eval()
    W.load_formula_weights(m, fam)
    x = torch.randn(2, 128, 8, 8, generator=gen_seed(128, 8))
    with torch.no_grad():
        save("residual_128", x=x, y=m(x))
    torch.manual_seed(0)
    m = ve.TransformerEncoderBlock(embed_dim=256, num_heads=8).eval()
    W.load_formula_weights(m, fam)
    x = torch.randn(2, 50, 256, generator=gen_seed(256, 50))
    with torch.no_grad():
        save("encblock_256_n50", x=x, y=m(x))
    # attention beyond the encoder's self-attention call: cross-attention (Lq != Lk), a key
    # padding mask and need_weights (manifold_layers.py:386-434)
    torch.manual_seed(0)
    m = ml.MultiHeadManifoldAttention(256, num_heads=8).eval()
    W.load_formula_weights(m, fam)
    q = torch.randn(2, 7, 256, generator=gen_seed(256, 7, 1))
    kv = torch.randn(2, 11, 256, generator=gen_seed(256, 11, 2))
    mask = torch.zeros(2, 11, dtype=torch.bool)
    mask[1, 8:] = True
    mask[0, ::3] = True
    with torch.no_grad():
        out, w = m(q, kv, kv, key_padding_mask=mask, need_weights=True)
        out_self, _ = m(q, q, q)
    save("attn_cross_mask", q=q, kv=kv, mask=mask, out=out, weights=w, out_self=out_self)
    # decoder on random logits
    dec = yh.YOLODecoder()
    ag = yh.YOLOAnchorGenerator()
    p = torch.randn(2, 3, 7, 9, 85, generator=gen_seed(85, 7)) * 2
    out = dec(p, ag(1), (13, 13))
    save("decode_s1", pred=p, boxes=out["boxes"], scores=out["scores"],
         class_scores=out["class_scores"], class_indices=out["class_indices"].to(torch.int16))


# ------------------------------------------------------------------ G4 full model
def top2_margin(scores: torch.Tensor) -> torch.Tensor:
    t = torch.topk(scores, 2, dim=-1).values
    return t[..., 0] - t[..., 1]


def gen_model(hv, only=None):
    print("G4 model")
    for tag, tiny, fam, S, B, sub in MODEL_CASES:
        if only and tag not in only:
            continue
        t0 = time.time()
        _TINY["on"] = tiny
        torch.manual_seed(0)
        model = hv.HybridVisionSystem({"image_size": S}).eval()
        _TINY["on"] = False
        W.load_formula_weights(model, fam)
        x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1))
        with torch.no_grad():
            out = model(x, task="detection")
            model64 = model.double()
            out64 = model64(x.double(), task="detection")
        rec = {"x_seed": 1, "B": B, "S": S, "tiny": int(tiny), "threads": torch.get_num_threads(),
               "sub": sub}
        for s in range(3):
            k = f"scale_{s}"
            pr = out["predictions"][k]
            pr64 = out64["predictions"][k]
            d = out["decoded"][k]
            d64 = out64["decoded"][k]
            step = sub if s == 0 else 1
            rec[f"pred{s}"] = pr[:, :, ::step]
            rec[f"pred{s}_f64"] = pr64[:, :, ::step].float()
            rec[f"cls{s}"] = d["class_indices"].to(torch.uint8)
            rec[f"cls{s}_f64"] = d64["class_indices"].to(torch.uint8)
            rec[f"margin{s}"] = top2_margin(d64["scores"]).float()
            rec[f"clsscore{s}"] = d["class_scores"]
            rec[f"boxes{s}"] = d["boxes"][:, :, ::step]
        rec["final_features"] = out["final_features"]
        rec["final_features_f64"] = out64["final_features"].float()
        rec["vit_features_pool"] = out["vit_features"].mean(dim=(2, 3))
        rec["fused_small_pool"] = out["fused_features"]["fused_small"].mean(dim=(2, 3))
        save(f"model_{tag}", **rec)
        print(f"  {tag}: {time.time() - t0:.1f}s")
        del model, model64


# ------------------------------------------------------------------ G5 training step
def gen_train(hv, only=None):
    """Training mode (BN batch statistics), every dropout p=0 so the step is deterministic,
    YOLOLoss on synthetic targets (hv_amd/targets.py builder), backward in fp32 and fp64.
    Records loss components, predictions, per-parameter gradient norms and gradient probes
    (<grad, fixed random direction>, oracle/cases.py:grad_probe), plus full gradients of a few
    small parameters.  Cases: oracle/cases.py TRAIN_CASES (tiny 64 B2; base 224 B2 = config C's
    model)."""
    print("G5 train")
    import json
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "humanoid-vision-system_amd"))
    from hv_amd.targets import synthetic_targets
    from oracle.cases import TRAIN_CASES, grad_probe
    for tag, tiny, S, B, tseed in TRAIN_CASES:
        if only and tag not in only:
            continue
        t0 = time.time()
        _TINY["on"] = tiny
        torch.manual_seed(0)
        model = hv.HybridVisionSystem({"image_size": S})
        _TINY["on"] = False
        W.load_formula_weights(model, "wc")
        for mod in model.modules():
            if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
                mod.p = 0.0
        x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1))
        tg = synthetic_targets(B, S, seed=tseed)
        rec = {"B": B, "S": S, "target_seed": tseed, "threads": torch.get_num_threads()}
        for sfx, dt in (("", torch.float32), ("_f64", torch.float64)):
            m = model.to(dt).train()
            m.zero_grad(set_to_none=True)
            out = m(x.to(dt), targets=[t.to(dt) for t in tg], compute_loss=True)
            loss = out["loss"]
            loss["total_loss"].backward()
            rec["total_loss" + sfx] = loss["total_loss"].detach().float()
            for k in ("coord_loss", "obj_loss", "noobj_loss", "cls_loss"):
                rec[k + sfx] = torch.tensor(float(loss[k]))
            for sidx in range(3):
                rec[f"pred{sidx}" + sfx] = out["predictions"][f"scale_{sidx}"].detach().float()
            names = [n for n, p in m.named_parameters()]
            rec["grad_norm" + sfx] = torch.tensor([p.grad.double().norm().item() if p.grad is not None else -1.0
                                                   for p in m.parameters()])
            rec["grad_probe" + sfx] = torch.tensor(
                [float(p.grad.double().flatten() @ grad_probe(n, p.numel())) / math.sqrt(p.numel())
                 if p.grad is not None else 0.0 for n, p in m.named_parameters()])
            for n, p in m.named_parameters():
                if p.grad is not None and p.numel() <= 4096 and ("norm_post" in n or "bn." in n or "H_res_raw" in n
                                                                  and p.numel() <= 1024 or "pred_conv.bias" in n):
                    rec["g:" + n + sfx] = p.grad.detach().float()
            del out, loss
        kind = "tiny" if tiny else "base"
        with open(os.path.join(OUT, f"train_{kind}_param_names.json"), "w") as f:
            json.dump(names, f)
        save(f"train_{tag}", **rec)
        print(f"  {tag}: {time.time() - t0:.1f}s")
        del model, m


# ------------------------------------------------------------------ G8 reference bf16 (S8)
def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-300))


def gen_bf16ref(ml, hv, parts):
    """The reference's OWN bf16 numerics (S8, oracle/autocast_emu.py: CUDA autocast's op policy
    emulated on CPU) on the fixtures' inputs, so that the HIP bf16 mode is held to a multiple of
    the error the reference itself makes in bf16 (instead of fixed bounds):
      mhc   -- every (D, e) of G2, both weight families, the reference's own autocast region
               (ManifoldHyperConnection.forward body, manifold_layers.py:247-263) in bf16;
      model -- base 640 B=2 eval (fixture model_base_wc_640_b2), the whole forward under the
               policy (the trainer's / engine's autocast region, mhc_trainer.py:241);
      train -- base 224 B=2 train step (fixture train_base_224_b2) under the policy, and base 640
               B=2 (config C's resolution; x seed 7, target seed 11) in fp32 AND under the policy
               (no fp64 at 640: the GPU test compares HIP bf16 with HIP fp32 there).
    Each record stores the reference-bf16 outputs' errors against the reference's fp64 (or fp32)
    run -- the anchors the GPU tests multiply."""
    from oracle.autocast_emu import CudaAutocastBF16, MhcOnly
    if "mhc" in parts:
        print("G8 mhc bf16ref")
        for fam in ("wc", "init"):
            for D, e in MHC_CASES:
                torch.manual_seed(0)
                m = ml.ManifoldHyperConnection(D, expansion_rate=e).eval()
                W.load_formula_weights(m, fam)
                x = mhc_input(D, e)
                g = np.load(os.path.join(OUT, f"mhc_{fam}_D{D}_e{e}.npz"))
                with torch.no_grad(), MhcOnly(ml):
                    yb = m(x)
                y64 = torch.from_numpy(g["y64"])
                rec = {"err_vs_f64": _rel(yb, y64), "maxabs_vs_f64": float((yb.double() - y64.double()).abs().max())}
                if D <= 512:
                    rec["y"] = yb
                save(f"mhc_{fam}_D{D}_e{e}_bf16ref", **rec)
                print(f"  {fam} D={D} e={e}: rel-L2 {rec['err_vs_f64']:.4f}")
    if "model" in parts:
        print("G8 model bf16ref")
        for tag, tiny, fam, S, B, sub in MODEL_CASES:
            if tag != "base_wc_640_b2":
                continue
            t0 = time.time()
            torch.manual_seed(0)
            model = hv.HybridVisionSystem({"image_size": S}).eval()
            W.load_formula_weights(model, fam)
            g = np.load(os.path.join(OUT, f"model_{tag}.npz"))
            x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1))
            with torch.no_grad(), CudaAutocastBF16() as mode:
                out = model(x, task="detection")
            rec = {"policy_counts": np.array([mode.counts["lower"], mode.counts["fp32"]])}
            agree = []
            for s in range(3):
                step = sub if s == 0 else 1
                pr = out["predictions"][f"scale_{s}"][:, :, ::step].float()
                bx = out["decoded"][f"scale_{s}"]["boxes"][:, :, ::step].float()
                rec[f"pred{s}_err_vs_f64"] = _rel(pr, torch.from_numpy(g[f"pred{s}_f64"]))
                rec[f"boxes{s}_err_vs_f32"] = _rel(bx, torch.from_numpy(g[f"boxes{s}"]))
                ci = out["decoded"][f"scale_{s}"]["class_indices"].numpy()
                sure = g[f"margin{s}"] >= 1e-2
                if sure.any():
                    agree.append(float((ci[sure] == g[f"cls{s}_f64"][sure]).mean()))
            rec["class_agreement_margin_1e-2"] = np.array(agree)
            ff = out["final_features"].float()
            rec["final_err_vs_f64"] = _rel(ff, torch.from_numpy(g["final_features_f64"]))
            save(f"model_{tag}_bf16ref", **rec)
            print(f"  {tag}: {time.time() - t0:.1f}s", {k: v for k, v in rec.items() if "err" in k}, agree)
    if "train" in parts:
        print("G8 train bf16ref")
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "humanoid-vision-system_amd"))
        from hv_amd.targets import synthetic_targets
        from oracle.cases import grad_probe

        def step(S, B, xseed, tseed, bf16, f64=False):
            torch.manual_seed(0)
            model = hv.HybridVisionSystem({"image_size": S})
            W.load_formula_weights(model, "wc")
            for mod in model.modules():
                if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
                    mod.p = 0.0
            model.train()
            x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(xseed))
            tg = synthetic_targets(B, S, seed=tseed)
            if f64:                      # as gen_train's fp64 run: fp32 weights and inputs, widened
                model = model.double()
                x, tg = x.double(), [t.double() for t in tg]
            if bf16:
                with CudaAutocastBF16():
                    out = model(x, targets=tg, compute_loss=True)
                    loss = out["loss"]
                    loss["total_loss"].float().backward()
            else:
                out = model(x, targets=tg, compute_loss=True)
                loss = out["loss"]
                loss["total_loss"].backward()
            r = {"total_loss": float(loss["total_loss"])}
            for k in ("coord_loss", "obj_loss", "noobj_loss", "cls_loss"):
                r[k] = float(loss[k])
            r["preds"] = [out["predictions"][f"scale_{s}"].detach().float() for s in range(3)]
            r["grad_norm"] = np.array([p.grad.double().norm().item() if p.grad is not None else -1.0
                                       for p in model.parameters()])
            r["grad_probe"] = np.array([float(p.grad.double().flatten() @ grad_probe(n, p.numel())) / math.sqrt(p.numel())
                                        if p.grad is not None else 0.0 for n, p in model.named_parameters()])
            return r

        t0 = time.time()
        g = np.load(os.path.join(OUT, "train_base_224_b2.npz"))
        if "train224seeds" in parts or "train640seeds" in parts:
            if "train224seeds" in parts:
                gen_train224_seeds(step, g)
            if "train640seeds" in parts:
                gen_train640_seeds(step)
            return
        r = step(int(g["S"]), int(g["B"]), 1, int(g["target_seed"]), True)
        rec = {k: np.float64(r[k]) for k in ("total_loss", "coord_loss", "obj_loss", "noobj_loss", "cls_loss")}
        rec["grad_norm"], rec["grad_probe"] = r["grad_norm"], r["grad_probe"]
        for s in range(3):
            rec[f"pred{s}_err_vs_f64"] = _rel(r["preds"][s], torch.from_numpy(g[f"pred{s}_f64"]))
        save("train_base_224_b2_bf16ref", **rec)
        print(f"  224: {time.time() - t0:.1f}s loss {rec['total_loss']:.5f} vs f64 {float(g['total_loss_f64']):.5f}")
        t0 = time.time()
        r32 = step(640, 2, 7, 11, False)
        r16 = step(640, 2, 7, 11, True)
        rec = {}
        for k in ("total_loss", "coord_loss", "obj_loss", "noobj_loss", "cls_loss"):
            rec[k + "_f32"], rec[k + "_bf16"] = np.float64(r32[k]), np.float64(r16[k])
        rec["grad_norm_f32"], rec["grad_norm_bf16"] = r32["grad_norm"], r16["grad_norm"]
        rec["grad_probe_f32"], rec["grad_probe_bf16"] = r32["grad_probe"], r16["grad_probe"]
        rec["logits_rel_l2_bf16_vs_f32"] = np.array([_rel(r16["preds"][s], r32["preds"][s]) for s in range(3)])
        save("train_base_640_b2_ref", **rec)
        print(f"  640: {time.time() - t0:.1f}s logits bf16 vs f32 {rec['logits_rel_l2_bf16_vs_f32']}")


def gen_train224_seeds(step, g):
    """The base 224 B=2 training step on two more input batches (x seeds 2, 3; the fixture's
    targets), in fp64 and under the bf16 policy: per-parameter gradient norms of both, so the GPU
    test compares gradient-group errors as a MEDIAN over three batches (seed 1 = the fixture) --
    at init this model's bf16 gradient groups are chaotic (any rounding difference is amplified
    through the ViT's backward), so one batch is one noisy sample of each group's error."""
    t0 = time.time()
    path = os.path.join(OUT, "train_base_224_b2_seeds.npz")
    rec = dict(np.load(path)) if os.path.exists(path) else {}
    for xs in TRAIN224_SEEDS:
        if f"grad_norm_bf16_s{xs}" in rec:
            continue
        r64 = step(int(g["S"]), int(g["B"]), xs, int(g["target_seed"]), False, f64=True)
        r16 = step(int(g["S"]), int(g["B"]), xs, int(g["target_seed"]), True)
        rec[f"grad_norm_f64_s{xs}"], rec[f"grad_norm_bf16_s{xs}"] = r64["grad_norm"], r16["grad_norm"]
        rec[f"total_loss_f64_s{xs}"], rec[f"total_loss_bf16_s{xs}"] = np.float64(r64["total_loss"]), \
            np.float64(r16["total_loss"])
        print(f"  224 seed {xs}: {time.time() - t0:.1f}s loss f64 {r64['total_loss']:.6f} bf16 {r16['total_loss']:.6f}")
        save("train_base_224_b2_seeds", **rec)


from oracle.cases import TRAIN224_SEEDS, TRAIN640_SEEDS  # noqa: E402


def gen_train640_seeds(step):
    """Config C's resolution on two more batches (x seeds 8, 9; targets 11), fp32 and under the
    bf16 policy: per-parameter gradient norms for the 640 anchor's median over three batches."""
    t0 = time.time()
    path = os.path.join(OUT, "train_base_640_b2_seeds.npz")
    rec = dict(np.load(path)) if os.path.exists(path) else {}
    for xs in TRAIN640_SEEDS:
        if f"grad_norm_bf16_s{xs}" in rec:
            continue
        r32 = step(640, 2, xs, 11, False)
        r16 = step(640, 2, xs, 11, True)
        rec[f"grad_norm_f32_s{xs}"], rec[f"grad_norm_bf16_s{xs}"] = r32["grad_norm"], r16["grad_norm"]
        rec[f"total_loss_f32_s{xs}"], rec[f"total_loss_bf16_s{xs}"] = np.float64(r32["total_loss"]), \
            np.float64(r16["total_loss"])
        print(f"  640 seed {xs}: {time.time() - t0:.1f}s")
        save("train_base_640_b2_seeds", **rec)


# ------------------------------------------------------------------ G6 post-processing
def gen_nms(yh):
    """YOLODetectionHead.post_process (yolo_head.py:571-731) on random decoded outputs."""
    print("G6 nms")
    from oracle.cases import nms_case
    torch.manual_seed(0)
    head = yh.YOLODetectionHead([16, 16, 16], num_classes=80)
    for seed, conf, iou, mx in ((1, 0.5, 0.5, 100), (2, 0.3, 0.4, 100), (3, 0.5, 0.5, 7), (4, 0.99, 0.5, 100)):
        dec = nms_case(seed)
        res = head.post_process(dec, confidence_threshold=conf, iou_threshold=iou, max_detections=mx)
        rec = {"conf": conf, "iou": iou, "max_det": mx}
        for b, r in enumerate(res):
            rec[f"boxes{b}"] = r["boxes"].reshape(-1, 4)
            rec[f"scores{b}"] = r["scores"].reshape(-1)
            rec[f"labels{b}"] = r["labels"].reshape(-1)
        save(f"nms_{seed}", **rec)


def gen_nms_large(yh):
    """post_process at detection-grid sizes past the GPU kernel's LDS capacity and max_det past
    1024 (oracle/cases.NMS_LARGE_CASES).  Inputs are regenerated from oracle/cases.nms_case."""
    print("G6b nms large")
    from oracle.cases import NMS_LARGE_CASES, nms_case
    torch.manual_seed(0)
    head = yh.YOLODetectionHead([16, 16, 16], num_classes=80)
    for tag, seed, B, grids, conf, iou, mx, spread in NMS_LARGE_CASES:
        dec = nms_case(seed, B=B, grids=grids, spread=spread)
        ncand = [int((v["class_scores"].reshape(B, -1) > conf).sum(1).max()) for _, v in sorted(dec.items())]
        res = head.post_process(dec, confidence_threshold=conf, iou_threshold=iou, max_detections=mx)
        rec = {"conf": conf, "iou": iou, "max_det": mx, "max_candidates": np.array(ncand)}
        for b, r in enumerate(res):
            rec[f"boxes{b}"] = r["boxes"].reshape(-1, 4)
            rec[f"scores{b}"] = r["scores"].reshape(-1)
            rec[f"labels{b}"] = r["labels"].reshape(-1)
        print(f"  {tag}: candidates per scale {ncand}, kept {[len(r['scores']) for r in res]}")
        save(f"nms_large_{tag}", **rec)


def gen_preproc():
    """G7: the reference's default preprocessing resize -- torchvision Resize on a PIL image,
    i.e. Pillow Image.resize(BILINEAR) (preprocessing.py:104-131,268-274; Pillow pinned 10.0.0 in
    requirements.txt, the same Resample.c algorithm as the Pillow installed here).  Stores the
    resized uint8 RGB images; inputs are regenerated from oracle/cases.camera_frames."""
    print("G7 preprocessing (Pillow)")
    import PIL
    from PIL import Image
    from oracle.cases import PIL_CASES, camera_frames
    for tag, n, h, w, oh, ow, seed in PIL_CASES:
        bgr = camera_frames(seed, n, h, w)
        outs = []
        for i in range(n):
            rgb = bgr[i][:, :, ::-1].copy()                      # cv2.cvtColor(BGR2RGB), preprocessing.py:202-205
            outs.append(np.asarray(Image.fromarray(rgb).resize((ow, oh), Image.BILINEAR)))
        save(f"preproc_pil_{tag}", seed=seed, in_hw=np.array([n, h, w]), out_hw=np.array([oh, ow]),
             resized_rgb=np.stack(outs), pillow_version=np.array(PIL.__version__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="sinkhorn,stability,mhc,blocks,model,layout,train,nms,preproc")
    ap.add_argument("--models", default="")
    ap.add_argument("--trains", default="")
    ap.add_argument("--bf16ref", default="mhc,model,train")
    a = ap.parse_args()
    torch.set_num_threads(8)
    ml, vb, ve, yh, hv = apply_shims()
    parts = a.only.split(",")
    if "sinkhorn" in parts:
        gen_sinkhorn(ml)
    if "stability" in parts:
        gen_stability(ml)
    if "mhc" in parts:
        gen_mhc(ml)
    if "mhc" in parts or "mhclarge" in parts:
        gen_mhc_large(ml)
    if "blocks" in parts:
        gen_blocks(ml, vb, ve, yh)
    if "model" in parts:
        gen_model(hv, [m for m in a.models.split(",") if m])
    if "layout" in parts:
        gen_layout(hv)
    if "train" in parts:
        gen_train(hv, [m for m in a.trains.split(",") if m])
    if "nms" in parts:
        gen_nms(yh)
    if "nms" in parts or "nmslarge" in parts:
        gen_nms_large(yh)
    if "preproc" in parts:
        gen_preproc()
    if "seeded" in parts:
        gen_seeded_init(hv)
    if "bf16ref" in parts:
        gen_bf16ref(ml, hv, [p for p in a.bf16ref.split(",") if p])



def gen_layout(hv):
    """Record the reference state_dict layout (names, shapes, dtypes) for tiny and base."""
    import json
    for tag, tiny in (("tiny", True), ("base", False)):
        _TINY["on"] = tiny
        torch.manual_seed(0)
        model = hv.HybridVisionSystem({})
        _TINY["on"] = False
        lay = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in model.state_dict().items()]
        path = os.path.join(OUT, f"state_dict_{tag}.json")
        with open(path, "w") as f:
            json.dump(lay, f)
        anchors = model.detection_head.anchor_generator.anchors
        np.save(os.path.join(OUT, "anchors.npy"), anchors.numpy())
        print(f"  wrote {path} ({len(lay)} entries)")


def gen_seeded_init(hv):
    """Parameter values of the reference model built right after torch.manual_seed(0)
    (hybrid_vision.py:53-197 and every submodule constructor: the RNG draws of each
    torch.randn / nn.Linear / nn.Conv2d default init before the explicit re-inits).  Per
    state_dict entry (state_dict_<tag>.json order): the first 8 and last 4 flattened values and
    the fp64 sum and sum of squares."""
    import json
    for tag, tiny in (("tiny", True), ("base", False)):
        _TINY["on"] = tiny
        torch.manual_seed(0)
        model = hv.HybridVisionSystem({})
        _TINY["on"] = False
        names = [k for k, _, _ in json.load(open(os.path.join(OUT, f"state_dict_{tag}.json")))]
        sd = model.state_dict()
        P = len(names)
        head = np.full((P, 8), np.nan, dtype=np.float32)
        tail = np.full((P, 4), np.nan, dtype=np.float32)
        s1 = np.zeros(P, dtype=np.float64)
        s2 = np.zeros(P, dtype=np.float64)
        for i, n in enumerate(names):
            v = sd[n].detach().reshape(-1)
            if not v.is_floating_point():
                v = v.double()
            v = v.double()
            head[i, :min(8, v.numel())] = v[:8].float().numpy()
            tail[i, :min(4, v.numel())] = v[-4:].float().numpy() if v.numel() else []
            s1[i] = float(v.sum())
            s2[i] = float((v * v).sum())
        save(f"seeded_init_{tag}", head=head, tail=tail, s1=s1, s2=s2)


if __name__ == "__main__":
    main()
