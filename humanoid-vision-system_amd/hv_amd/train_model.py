"""HybridVisionSystem forward in training mode, built from the autograd
Functions of train_fn.py.  It walks the same modules (and parameters) as the inference path,
in the reference's order (hybrid_vision.py:222-367), with BatchNorm batch statistics,
dropout and every backward on hand-written HIP kernels.

Layout: NHWC / token-major activations in the compute dtype (bf16 or fp32), fp32 parameters
and gradients.  All 76 Sinkhorn projections run as ONE grouped autograd node
(SinkhornGroupFn) whose backward is one grouped reverse sweep.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from . import ops_train as OT
from . import train_fn as TF
from .layers import to_nchw_view, to_nhwc
from .manifold import flush_stability
from .runtime import PRECISIONS


class HTable(dict):
    """id(mHC) -> its differentiable H_res (this forward's grouped Sinkhorn output); `coefs` holds
    the sites' grouped training coefficients (train_prep.TrainCoef) when they were prepared."""
    coefs: Dict[int, Any] = {}


class _InFlight:
    """Marks one cached (Sinkhorn group, coefficient prep) set as used by a forward whose backward
    has not run yet: a second training forward before that backward (`model(x1) + model(x2)`,
    checkpoint-style recomputation) must not overwrite the buffers the first one's backward
    reads, so it takes another set.  Released by SinkhornGroupFn.backward, or when the forward's
    autograd graph is dropped without a backward (the token lives in its ctx)."""

    def __init__(self, entry: Dict):
        self.entry = entry
        entry["busy"] += 1

    def release(self) -> None:
        if self.entry is not None:
            self.entry["busy"] -= 1
            self.entry = None

    def __del__(self):
        self.release()


def _hres_table(model) -> HTable:
    """Grouped differentiable Sinkhorn of all 76 sites + (model.hv_train_group_prep, default on)
    the grouped training coefficient prep of train_prep.TrainPrep over its outputs.  The Sinkhorn
    group and the prep program are cached on the model while the parameter storage is unchanged,
    so their buffers (and a captured training graph's pointers) stay put.  The cache is a small
    pool: a forward whose set is still waiting for its backward leaves it alone (_InFlight)."""
    from .train_prep import TrainPrep
    mods = model._mhc_modules
    raws = [m.H_res_raw for m in mods]
    dt = PRECISIONS[model.hv_precision]
    cache = model.__dict__.setdefault("_train_prep_cache", {})
    key = (tuple(r.data_ptr() for r in raws), tuple(m.sinkhorn.convergence_history.data_ptr() for m in mods))
    pool = [e for e in cache.get("pool", []) if e["key"] == key]
    cache["pool"] = pool
    entry = next((e for e in pool if e["busy"] == 0), None)
    if entry is None:
        group = ops.SinkhornGroup([r.detach() for r in raws], [m.sinkhorn.num_iterations for m in mods],
                                  raws[0].device, mods[0].sinkhorn.epsilon, mods[0].sinkhorn.tau,
                                  hists=[m.sinkhorn.convergence_history for m in mods])
        entry = {"key": key, "sk": group, "prep": None, "busy": 0}
        pool.append(entry)
    token = _InFlight(entry) if torch.is_grad_enabled() else None
    outs = TF.SinkhornGroupFn.apply(entry["sk"], token, *raws)
    H = HTable({id(m): h for m, h in zip(mods, outs)})
    H.coefs = {}
    if getattr(model, "hv_train_group_prep", True):
        prep = entry["prep"]
        if prep is None or not prep.valid_for(mods, outs, dt):
            prep = entry["prep"] = TrainPrep(mods, [o.detach() for o in outs], dt)
        H.coefs = prep.run()
    return H


def _mhc(m, x: torch.Tensor, H, out_f32: bool = False) -> torch.Tensor:
    """TF.mhc with the site's grouped coefficients when the table carries them."""
    return TF.mhc(m, x, H[id(m)], getattr(H, "coefs", {}).get(id(m)), out_f32)


def module_H(module) -> Dict[int, torch.Tensor]:
    """Grouped differentiable Sinkhorn projections of every mHC inside `module` (module-level
    training calls; the system forward builds one table for all 76 sites)."""
    from .manifold import ManifoldHyperConnection
    mods = [m for m in module.modules() if isinstance(m, ManifoldHyperConnection)]
    if not mods:
        return {}
    raws = [m.H_res_raw for m in mods]
    group = ops.SinkhornGroup([r.detach() for r in raws], [m.sinkhorn.num_iterations for m in mods],
                              raws[0].device, mods[0].sinkhorn.epsilon, mods[0].sinkhorn.tau,
                              hists=[m.sinkhorn.convergence_history for m in mods])
    outs = TF.SinkhornGroupFn.apply(group, None, *raws)
    return {id(m): h for m, h in zip(mods, outs)}


def nhwc_in(x: torch.Tensor, dtype) -> torch.Tensor:
    """Differentiable NCHW -> contiguous NHWC in the compute dtype (module-entry glue)."""
    return x.permute(0, 2, 3, 1).contiguous().to(dtype)


def _tok(m, x: torch.Tensor, H) -> torch.Tensor:
    n, h, w, c = x.shape
    return _mhc(m, x.reshape(-1, c), H).view(n, h, w, c)


def _dropout2d(x: torch.Tensor, p: float) -> torch.Tensor:
    """nn.Dropout2d on NHWC: one keep/scale per (image, channel)."""
    if p <= 0:
        return x
    n, c = x.shape[0], x.shape[-1]
    mask = OT.dropout(torch.ones((n, c), device=x.device, dtype=torch.float32), p, TF.next_seed())
    return _ChannelScaleFn.apply(x, mask)


class _ChannelScaleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask):
        ctx.save_for_backward(mask)
        return ops.scale_residual(x.contiguous(), mask, None)

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        return ops.scale_residual(g.contiguous(), mask, None), None


# ------------------------------------------------------------------------- backbone
def conv_mhc_layer(l, x, H, extra_residual=None):
    """ConvMHCLayer.forward (vision_backbone.py:99-134) in training mode."""
    y = TF.conv(x, l.conv, l.bn, l.act_name)
    if l.mhc is not None:
        y = _tok(l.mhc, y, H)
        if l.channel_attention is not None:
            ca = l.channel_attention
            y = TF.SEGateFn.apply(y, x if l.use_residual else None, ca[1].weight, ca[1].bias, ca[3].weight, ca[3].bias)
            if extra_residual is not None:
                y = TF.AddFn.apply(y, extra_residual, 1.0)
            return y
    if l.use_residual:
        y = TF.AddFn.apply(y, x, 1.0)
    if extra_residual is not None:
        y = TF.AddFn.apply(y, extra_residual, 1.0)
    return y


def residual_layer(r, x, H):
    y = x
    for b in r.blocks:
        y = conv_mhc_layer(b, y, H)
    if isinstance(r.projection, nn.Identity):
        return TF.AddFn.apply(y, x, 1.0)
    return conv_mhc_layer(r.projection, y, H, extra_residual=x)


def backbone(bb, x, H):
    """HybridVisionBackbone.forward (vision_backbone.py:329-397)."""
    from .backbone import ConvMHCLayer
    for lyr in list(bb.stem)[:3]:
        x = conv_mhc_layer(lyr, x, H)
    x = TF.MaxPoolFn.apply(x)
    raw = {"stem": x}
    for i, st in enumerate(bb.stages):
        for lyr in st:
            x = conv_mhc_layer(lyr, x, H) if isinstance(lyr, ConvMHCLayer) else residual_layer(lyr, x, H)
        raw[f"stage_{i + 1}"] = x
    p = bb.dropout.p if isinstance(bb.dropout, nn.Dropout2d) else 0.0

    def enh(mod, f):
        return f if isinstance(mod, nn.Identity) else _tok(mod, f, H)

    return {"scale_small": _dropout2d(enh(bb.enhance_small, raw["stage_2"]), p),
            "scale_medium": _dropout2d(enh(bb.enhance_medium, raw["stage_3"]), p),
            "scale_large": _dropout2d(enh(bb.enhance_large, raw["stage_4"]), p),
            "raw_features": raw}


# ------------------------------------------------------------------------- transformer
def _positions(pe: torch.Tensor, tokens: int) -> torch.Tensor:
    """[1, L+1, D] table -> [tokens+1, D] (shim S3: linear interpolation of the patch slots)."""
    t = pe[0]
    if t.shape[0] == tokens + 1:
        return t
    body = F.interpolate(t[1:].t().unsqueeze(0), size=(tokens,), mode="linear").squeeze(0).t()
    return torch.cat([t[:1], body], dim=0)


def attention(a, x, n, H):
    """MultiHeadManifoldAttention.forward (manifold_layers.py:386-434) on x [n*L, D]."""
    L = x.shape[0] // n
    q = _mhc(a.q_proj, x, H).view(n, L, -1)
    k = _mhc(a.k_proj, x, H).view(n, L, -1)
    v = _mhc(a.v_proj, x, H).view(n, L, -1)
    p = a.dropout.p
    o = TF.AttentionFn.apply(q, k, v, a.num_heads, p, TF.next_seed() if p > 0 else 0)
    return _mhc(a.out_proj, o.reshape(n * L, -1), H)


VIT_F32_STREAM = True     # tools/vit_grad_probe.py A/B switch: the ViT residual stream in fp32


def encoder_block(blk, x, n, H, dt):
    """TransformerEncoderBlock.forward (vit_encoder_decoder.py:174-210).  The residual stream x is
    fp32 in every precision, as under the reference's autocast: the residual mHC outputs are
    LayerNorm outputs (fp32 under autocast) and the adds of fp32 tensors stay fp32, so the stream
    -- and, in the backward, the gradient that flows down it through all blocks -- is never
    rounded to bf16; only the operands of the GEMMs (the RMSNorm outputs) are `dt`."""
    f32 = x.dtype == torch.float32
    h = TF.RMSNormFn.apply(x, blk.norm1.scale, blk.norm1.eps, dt)
    a = attention(blk.attention, h, n, H)
    a = _mhc(blk.residual_mhc1, a, H, out_f32=f32)
    p = blk.dropout.p
    x = TF.DropAddFn.apply(x, a, p, TF.next_seed() if p > 0 else 0)
    h = TF.RMSNormFn.apply(x, blk.norm2.scale, blk.norm2.eps, dt)
    h = TF.linear(h, blk.mlp[0], act="gelu", p=blk.mlp[2].p)
    h = TF.linear(h, blk.mlp[3], act="none", p=blk.mlp[4].p)
    h = _mhc(blk.residual_mhc2, h, H, out_f32=f32)
    return TF.DropAddFn.apply(x, h, p, TF.next_seed() if p > 0 else 0)


def vit_encoder(enc, x, H, features=None, head: bool = True):
    """VisionTransformerEncoder.forward (vit_encoder_decoder.py:277-315) -> CLS [n, D];
    `features` (a list) receives the token tensors after the embedding and every block."""
    pe = enc.patch_embed
    t = TF.conv(x, pe.projection)
    n, h, w, d = t.shape
    t = _mhc(pe.mhc_enhance, t.reshape(-1, d), H).view(n, h * w, d)
    pos = _positions(pe.position_embeddings, h * w)
    z = TF.VitAssembleFn.apply(t, pe.cls_token, pos)
    L = h * w + 1
    dt = z.dtype
    t = TF.RMSNormFn.apply(z.view(n * L, d), pe.norm.scale, pe.norm.eps,
                           torch.float32 if VIT_F32_STREAM else dt)          # the fp32 residual stream
    if features is not None:
        features.append(t.view(n, L, d))
    for blk in enc.blocks:
        t = encoder_block(blk, t, n, H, dt)
        if features is not None:
            features.append(t.view(n, L, d))
    cls = TF.GatherRowsFn.apply(t, L)
    cls = TF.RMSNormFn.apply(cls, enc.norm.scale, enc.norm.eps, dt)
    if head and isinstance(enc.head, nn.Linear):
        cls = TF.linear(cls, enc.head)
    return cls


def hybrid_encoder(he, cnn, H):
    """HybridVisionEncoder.forward (vit_encoder_decoder.py:470-520), shims S2/S3."""
    n, h, w, c = cnn.shape
    pe = he.pos_embed[0]
    pos = pe if pe.shape[0] == h * w else F.interpolate(pe.t().unsqueeze(0), size=(h * w,),
                                                        mode="linear").squeeze(0).t()
    v = _LinearPosFn.apply(cnn.reshape(-1, c), he.cnn_to_vit.weight, he.cnn_to_vit.bias, pos, h * w)
    v = v.view(n, h, w, -1)
    cls = vit_encoder(he.vit_encoder, v, H)                               # [n, D]
    e = TF.linear(cls, _Conv1x1AsLinear(he.vit_to_cnn), out_dtype=torch.float32)
    fused = TF.AddRowvecFn.apply(cnn, e)
    return _tok(he.fusion_mhc, fused, H)


class _Conv1x1AsLinear:
    """View a 1x1 Conv2d as a Linear (weight [cout, cin, 1, 1] -> [cout, cin]) for TF.linear."""

    def __init__(self, conv):
        self.weight = conv.weight.view(conv.weight.shape[0], -1)
        self.bias = conv.bias


class _LinearPosFn(torch.autograd.Function):
    """1x1 conv + bias + learned positional table broadcast over images, as one GEMM epilogue
    (vit_encoder_decoder.py:485-499): y[n*hw + p] = x W^T + b + pos[p]."""

    @staticmethod
    def forward(ctx, x, weight, bias, pos, hw: int):
        dt = x.dtype
        w = ops.cast(weight.detach().reshape(weight.shape[0], -1).float().contiguous(), dt)
        y = ops.gemm(x, w, bias=bias.detach().float().contiguous(), residual=pos.detach().float().contiguous(),
                     residual_mod=hw)
        ctx.hw = hw
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        g = g.contiguous()
        dt = x.dtype
        w2 = weight.detach().reshape(weight.shape[0], -1)
        dx = ops.gemm(g, OT.transpose_cast(w2, dt))
        dw = OT.wgrad(g, x).view_as(weight)
        db = OT.colsum(g)
        n = g.shape[0] // ctx.hw
        dpos = OT.colsum(g.view(n, ctx.hw * g.shape[1])).view(ctx.hw, g.shape[1])
        return dx, dw, db, dpos, None


# ------------------------------------------------------------------------- FPN + head
def fpn(f, feats, H):
    """FeaturePyramidNetwork.forward (feature_fusion.py:82-153)."""
    def refine(i, x):
        r = f.refinement_convs[i]
        x = TF.conv(x, r[0], r[1], "relu")
        x = TF.conv(x, r[3], r[4], "relu")
        return _tok(f.mhc_fusions[i], x, H)

    pl = TF.conv(feats["scale_large"], f.lateral_convs[2])
    pm = TF.conv(feats["scale_medium"], f.lateral_convs[1])
    ps = TF.conv(feats["scale_small"], f.lateral_convs[0])
    rl = refine(2, pl)
    out = {"fused_large": TF.conv(rl, f.output_convs[2])}
    rm = refine(1, TF.UpsampleAddFn.apply(pm, rl))
    out["fused_medium"] = TF.conv(rm, f.output_convs[1])
    rs = refine(0, TF.UpsampleAddFn.apply(ps, rm))
    out["fused_small"] = TF.conv(rs, f.output_convs[0])
    return out


def head_logits(ph, x, H):
    """YOLOPredictionHead.forward up to the 1x1 prediction conv (yolo_head.py:170-195), NHWC."""
    c = ph.conv_layers
    x = TF.conv(x, c[0], c[1], "leaky")
    x = TF.conv(x, c[3], c[4], "leaky")
    if not isinstance(ph.mhc_enhance, nn.Identity):
        x = _tok(ph.mhc_enhance, x, H)
    return TF.conv(x, ph.pred_conv)


# ------------------------------------------------------------------------- system
def system_forward(model, x: torch.Tensor, targets=None, task: str = "detection",
                   compute_loss: bool = False) -> Dict[str, Any]:
    """HybridVisionSystem.forward(x, targets, task, compute_loss) with model.training True.
    The model's HVOptions (kernel variants) apply to this forward and its backward
    (runtime._TRAIN during the forward; runtime.carry_train_state hands them to the backward, which
    runs on autograd's worker thread outside any RunCtx)."""
    from .runtime import _TRAIN, module_options
    prev = _TRAIN.opts
    _TRAIN.opts = module_options(model)     # this forward only: every Function carries it into its backward
    try:
        return _system_forward(model, x, targets, task, compute_loss)
    finally:
        _TRAIN.opts = prev


def _system_forward(model, x: torch.Tensor, targets, task: str, compute_loss: bool) -> Dict[str, Any]:
    dt = PRECISIONS[model.hv_precision]
    H = _hres_table(model)
    xin = to_nhwc(x.detach(), dt)
    bb = backbone(model.backbone, xin, H)
    out: Dict[str, Any] = {}
    if model.use_vit:
        vit = hybrid_encoder(model.vit_encoder, bb["scale_large"], H)
        bb["scale_large"] = TF.AddFn.apply(bb["scale_large"], vit, 0.5)
        out["vit_features"] = to_nchw_view(vit)
    fused = fpn(model.feature_fusion, bb, H)
    head = model.detection_head
    if task == "detection":
        preds, decoded, logits, dets = {}, {}, {}, {}
        for s, key in enumerate(("fused_small", "fused_medium", "fused_large")):
            lg = head_logits(head.pred_heads[s], fused[key], H)
            logits[s] = lg
            awh = head.anchor_generator.anchors[s].reshape(head.num_anchors, 4)[:, 2:4].contiguous()
            with torch.no_grad():
                dec, pred = ops.yolo_decode(lg.detach(), head.num_anchors, head.num_classes, awh, detections=True)
            dets[("small_scale", "medium_scale", "large_scale")[s]] = dec.pop("detections")
            preds[f"scale_{s}"] = _PredViewFn.apply(lg, head.num_anchors) if lg.requires_grad else pred
            decoded[f"scale_{s}"] = dec
        out["predictions"] = preds
        out["decoded"] = decoded
        out["detections"] = dets
        if compute_loss and targets is not None:
            out["loss"] = yolo_loss(head.loss_fn, logits, targets, head.num_anchors)
            w = float(getattr(model, "hv_manifold_weight", 0.0))
            if w > 0:
                # the reference trainer's total (mhc_trainer.py:248-255): det + manifold_weight * reg
                reg = manifold_regularization(H)
                out["loss"]["manifold_loss"] = reg.detach()
                out["loss"]["total_loss"] = out["loss"]["total_loss"] + w * reg
    out["final_features"] = final_features(model, fused, H)
    bbv = {k: to_nchw_view(v) for k, v in bb.items() if k != "raw_features"}
    bbv["raw_features"] = {k: to_nchw_view(v) for k, v in bb["raw_features"].items()}
    out["backbone_features"] = bbv
    out["fused_features"] = {k: to_nchw_view(v) for k, v in fused.items()}
    flush_stability()              # this forward's monitored sites: one grouped eigensolve
    return out


def manifold_regularization(H: Dict[int, torch.Tensor]) -> torch.Tensor:
    """ManifoldConstrainedTrainer._compute_manifold_regularization (mhc_trainer.py:299-340), as
    intended (the committed call passes kwargs SinkhornKnoppProjection does not take):
    over every mHC site, with H = SK(H_res_raw) -- here the SAME differentiable projections the
    forward used (the grouped Sinkhorn), so the gradient flows through its grouped backward --
    mean|rowsum(H) - 1| + mean|colsum(H) - 1| + 0.1 mean relu(eigvalsh(H) - 1), averaged over the
    sites.  eigvalsh reads H's lower triangle as torch.linalg.eigvalsh does (the reference calls it
    on the unsymmetrised projection)."""
    terms = []
    for h in H.values():
        h2 = h if h.dim() == 2 else h.reshape(h.shape[-2], h.shape[-1])
        row = (h2.sum(1) - 1.0).abs().mean()
        col = (h2.sum(0) - 1.0).abs().mean()
        ev = torch.linalg.eigvalsh(h2)
        terms.append(row + col + 0.1 * F.relu(ev - 1.0).mean())
    return torch.stack(terms).mean()


class _PredViewFn(torch.autograd.Function):
    """NHWC logits [n, h, w, A*P] -> reference predictions [n, A, h, w, P] fp32 (differentiable)."""

    @staticmethod
    def forward(ctx, lg, A: int):
        n, h, w, ap = lg.shape
        ctx.meta = (lg.dtype, A)
        return lg.float().view(n, h, w, A, ap // A).permute(0, 3, 1, 2, 4).contiguous()

    @staticmethod
    def backward(ctx, g):
        dt, A = ctx.meta
        n, A_, h, w, P = g.shape
        return g.permute(0, 2, 3, 1, 4).reshape(n, h, w, A * P).to(dt).contiguous(), None


def yolo_loss(loss_fn, logits: Dict[int, torch.Tensor], targets, A: int) -> Dict[str, Any]:
    """YOLOLoss.forward (yolo_head.py:374-465) on the NHWC logits of every scale; the raw
    component sums are device tensors (no host sync), total_loss is differentiable."""
    lam = (loss_fn.lambda_coord, loss_fn.lambda_obj, loss_fn.lambda_noobj, loss_fn.lambda_cls)
    total = None
    comps = torch.zeros(4, device=logits[0].device, dtype=torch.float32)
    for s in range(loss_fn.num_scales):
        if s not in logits:
            continue
        contrib, sums = TF.YoloLossFn.apply(logits[s], targets[s], A, lam)
        comps = comps + sums[:4]
        total = contrib if total is None else total + contrib
    return {"coord_loss": comps[0], "obj_loss": comps[1], "noobj_loss": comps[2], "cls_loss": comps[3],
            "total_loss": total}


def final_features(model, fused, H):
    """_extract_final_features (hybrid_vision.py:369-402): GAP x3 -> cat -> mHC -> MLP, kept
    in the autograd graph as in the reference: a loss on final_features trains final_fusion
    and output_projection (the detection loss does not reach them, so they get no gradient)."""
    pooled = [_ChannelMeanFn.apply(fused[k]) for k in ("fused_small", "fused_medium", "fused_large")]
    dt = fused["fused_small"].dtype
    ff = model.final_fusion
    c = _CatCastFn.apply(dt, *pooled)
    c = TF.MhcFn.apply(c, H[id(ff)], ff.H_pre_raw, ff.H_post_raw, ff.norm_pre.weight, ff.norm_pre.bias,
                       ff.mlp[0].weight, ff.mlp[0].bias, ff.mlp[3].weight, ff.mlp[3].bias, ff.norm_post.weight,
                       ff.norm_post.bias, ff,
                       tuple(TF.next_seed() if p > 0 else 0 for p in (ff.mlp[2].p, ff.mlp[5].p, ff.dropout.p)))
    h = TF.LinearFn.apply(c, model.output_projection[2].weight, model.output_projection[2].bias, "relu", 0.0, 0,
                          None)
    return TF.LinearFn.apply(h, model.output_projection[4].weight, model.output_projection[4].bias, "none", 0.0,
                             0, torch.float32)


class _ChannelMeanFn(torch.autograd.Function):
    """Global average pool of an NHWC map -> fp32 [n, c] (hv_channel_mean); backward spreads
    g / (h*w) over the pixels."""

    @staticmethod
    def forward(ctx, x):
        ctx.meta = (x.shape, x.dtype)
        return ops.channel_mean(x.contiguous())

    @staticmethod
    def backward(ctx, g):
        shape, dt = ctx.meta
        n, c = shape[0], shape[-1]
        hw = 1
        for d in shape[1:-1]:
            hw *= d
        zero = torch.zeros(shape, device=g.device, dtype=dt)
        return ops.add_rowvec(zero, (g / hw).contiguous())


class _CatCastFn(torch.autograd.Function):
    """cat(pooled, dim 1) in the compute dtype (the [n, 1792] final-fusion input)."""

    @staticmethod
    def forward(ctx, dt, *xs):
        ctx.widths = [x.shape[1] for x in xs]
        return torch.cat(xs, 1).to(dt).contiguous()

    @staticmethod
    def backward(ctx, g):
        g = g.float()
        outs, o = [], 0
        for w in ctx.widths:
            outs.append(g[:, o:o + w].contiguous())
            o += w
        return (None, *outs)


def yolo_loss_api(loss_fn, predictions: Dict[str, torch.Tensor], targets) -> Dict[str, Any]:
    """YOLOLoss.forward on reference-layout predictions [B, A, H, W, 5+C] (training API)."""
    logits = {}
    A = None
    for s in range(loss_fn.num_scales):
        p = predictions.get(f"scale_{s}")
        if p is None:
            continue
        B, A, h, w, P = p.shape
        logits[s] = p.permute(0, 2, 3, 1, 4).reshape(B, h, w, A * P).contiguous()
    return yolo_loss(loss_fn, logits, targets, A)


from .runtime import carry_train_state  # noqa: E402

carry_train_state(globals())
