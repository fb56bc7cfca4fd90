"""CPU restatement of the reference HybridVision forward path (the parity ORACLE).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker /
the timed CPU baseline -- never as part of the shipped product path.

This is a from-scratch functional restatement (plain torch CPU ops over a state_dict
that uses the reference's parameter names) of the semantics fixed in SURVEY.md §0.2:
the reference code plus shims S1-S7.  Every function cites the reference file:line it
follows.  It runs in float32 (the reference dtype) or float64.

It is pinned by ``tests/golden/*.npz``, produced by ``oracle/gen_golden.py`` which
imports the reference itself (read-only) with the shims applied
(``tests/test_oracle_golden.py``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

DEFAULT_ANCHORS = [
    [(10, 13), (16, 30), (33, 23)],
    [(30, 61), (62, 45), (59, 119)],
    [(116, 90), (156, 198), (373, 326)],
]


@dataclass
class OracleConfig:
    """Architecture knobs. Defaults = reference (hybrid_vision.py:54-74, manifold_layers.py:135)."""
    num_blocks: List[int] = field(default_factory=lambda: [2, 3, 4, 2])
    vit_depth: int = 6
    sk_iters: int = 20
    num_classes: int = 80
    base_channels: int = 32


TINY = OracleConfig(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5)
BASE = OracleConfig()


# ----------------------------------------------------------------------------------------
# a1: Sinkhorn-Knopp (manifold_layers.py:32-93, shim S1 for 2-D input)
# ----------------------------------------------------------------------------------------
def sinkhorn(raw: Tensor, iters: int, eps: float = 1e-8, tau: float = 1.0,
             history: Optional[Tensor] = None) -> Tensor:
    """softmax(raw/tau, -1)*m then ``iters`` x (row-normalise, column-normalise).

    manifold_layers.py:56-57 (init), :64-73 (iterations), :76-77 (history = |mean(row_sum)-1|).
    Accepts [n, m] (S1: treated as a batch of one) or [B, n, m].
    """
    squeeze = raw.dim() == 2
    m3 = raw.unsqueeze(0) if squeeze else raw
    m = m3.shape[-1]
    mat = torch.softmax(m3 / tau, dim=-1) * m
    for i in range(iters):
        rs = mat.sum(dim=2, keepdim=True)
        mat = mat / (rs + eps)
        cs = mat.sum(dim=1, keepdim=True)
        mat = mat / (cs + eps)
        if history is not None:
            history[i] = (rs.mean() - 1.0).abs()
    return mat.squeeze(0) if squeeze else mat


# ----------------------------------------------------------------------------------------
# a4: stability monitor (manifold_layers.py:282-316), fp64
# ----------------------------------------------------------------------------------------
def monitor_stability(H: Tensor, x_in: Tensor, x_out: Tensor) -> Dict[str, Tensor]:
    """eigenvalues of (H + H^T)/2 ascending (:288-290, eigvalsh), signal ratio
    mean|x_out| / (mean|x_in| + 1e-8) over the last dim (:296-298), |mean row/col sum - 1|
    (:306-315).  Computed in fp64 from the given fp32 tensors."""
    h = H.double()
    ev = torch.linalg.eigvalsh((h + h.T) / 2)
    ratio = x_out.double().norm(dim=-1).mean() / (x_in.double().norm(dim=-1).mean() + 1e-8)
    return {"eigenvalues": ev, "signal_ratio": ratio,
            "row_sum_error": (h.sum(dim=1).mean() - 1.0).abs(),
            "col_sum_error": (h.sum(dim=0).mean() - 1.0).abs()}


# ----------------------------------------------------------------------------------------
# a2/a3: mHC layer (manifold_layers.py:205-280), eval mode (dropout = identity)
# ----------------------------------------------------------------------------------------
def mhc_coefficients(sd: Dict[str, Tensor], p: str, sk_iters: int):
    """constrained_matrices (manifold_layers.py:205-221)."""
    H_pre = torch.sigmoid(sd[p + "H_pre_raw"])
    H_post = 2.0 * torch.sigmoid(sd[p + "H_post_raw"])
    H_res = sinkhorn(sd[p + "H_res_raw"], sk_iters)
    return H_pre, H_post, H_res


def mhc(sd: Dict[str, Tensor], p: str, x: Tensor, sk_iters: int) -> Tensor:
    """ManifoldHyperConnection.forward on token-major x[..., D] (manifold_layers.py:223-280)."""
    shape = x.shape
    D = shape[-1]
    x2 = x.reshape(-1, D)
    H_pre, H_post, H_res = mhc_coefficients(sd, p, sk_iters)
    xn = F.layer_norm(x2, (D,), sd[p + "norm_pre.weight"], sd[p + "norm_pre.bias"], 1e-5)
    e = xn @ H_pre                                                           # :253
    h = F.gelu(F.linear(e, sd[p + "mlp.0.weight"], sd[p + "mlp.0.bias"]))    # :163-165
    h = F.gelu(F.linear(h, sd[p + "mlp.3.weight"], sd[p + "mlp.3.bias"]))    # :167-168
    y = x2 @ H_res + h @ H_post                                              # :259-264
    y = F.layer_norm(y, (D,), sd[p + "norm_post.weight"], sd[p + "norm_post.bias"], 1e-5)
    return y.reshape(shape)


def mhc_nchw(sd, p, x: Tensor, sk_iters: int) -> Tensor:
    """Channels-last application on an NCHW map (vision_backbone.py:118-123; shim S2)."""
    return mhc(sd, p, x.permute(0, 2, 3, 1), sk_iters).permute(0, 3, 1, 2)


def rmsnorm(x: Tensor, scale: Tensor, eps: float = 1e-8) -> Tensor:
    """RMSNorm (manifold_layers.py:449-456)."""
    rms = torch.sqrt(torch.mean(x.pow(2), dim=-1, keepdim=True) + eps)
    return x / rms * scale


_BN_TRAIN = {"on": False}


class train_mode:
    """Within this context BatchNorm uses batch statistics (nn.BatchNorm2d in training mode,
    vision_backbone.py:113 / feature_fusion.py:44 / yolo_head.py:122); dropout stays off, so the
    training forward is deterministic and comparable (autograd of this restatement is the
    gradient oracle of the training step)."""

    def __enter__(self):
        _BN_TRAIN["on"] = True

    def __exit__(self, *exc):
        _BN_TRAIN["on"] = False
        return False


def batchnorm_eval(x: Tensor, sd, p: str, eps: float = 1e-5) -> Tensor:
    if _BN_TRAIN["on"]:
        return F.batch_norm(x, None, None, sd[p + "weight"], sd[p + "bias"], True, 0.0, eps)
    return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"],
                        sd[p + "weight"], sd[p + "bias"], False, 0.0, eps)


def yolo_loss(preds: Dict[str, Tensor], targets: List[Tensor], lambdas=(5.0, 1.0, 0.5, 1.0)):
    """YOLOLoss.forward (yolo_head.py:374-465): per scale, skipped without objects; coordinate
    MSE, BCE-with-logits obj/noobj/cls, each sum divided by that scale's object count."""
    lc, lo, ln, lcl = lambdas
    total = 0.0
    comps = {"coord_loss": 0.0, "obj_loss": 0.0, "noobj_loss": 0.0, "cls_loss": 0.0}
    for s in range(len(targets)):
        pred, tgt = preds[f"scale_{s}"], targets[s]
        obj = tgt[..., 4] > 0.5
        noobj = tgt[..., 4] < 0.5
        n = int(obj.sum())
        if n == 0:
            continue
        coord = F.mse_loss(pred[obj][:, :4], tgt[obj][:, :4], reduction="sum")
        o = F.binary_cross_entropy_with_logits(pred[obj][:, 4:5], tgt[obj][:, 4:5], reduction="sum")
        no = F.binary_cross_entropy_with_logits(pred[noobj][:, 4:5], tgt[noobj][:, 4:5], reduction="sum")
        c = F.binary_cross_entropy_with_logits(pred[obj][:, 5:], tgt[obj][:, 5:], reduction="sum")
        comps["coord_loss"] += float(coord.detach())
        comps["obj_loss"] += float(o.detach())
        comps["noobj_loss"] += float(no.detach())
        comps["cls_loss"] += float(c.detach())
        total = total + (lc * coord + lo * o + ln * no + lcl * c) / n
    comps["total_loss"] = total
    return comps


# ----------------------------------------------------------------------------------------
# a7-a9: CNN backbone (vision_backbone.py)
# ----------------------------------------------------------------------------------------
def conv_mhc_layer(sd, p: str, x: Tensor, cin: int, cout: int, k: int, stride: int,
                   sk_iters: int) -> Tensor:
    """ConvMHCLayer.forward (vision_backbone.py:99-134), use_mhc=True, SiLU."""
    identity = x
    y = F.conv2d(x, sd[p + "conv.weight"], None, stride, k // 2)
    y = F.silu(batchnorm_eval(y, sd, p + "bn."))
    y = mhc_nchw(sd, p + "mhc.", y, sk_iters)
    if cout >= 32:                                  # SE gate :76-85,126-128
        g = y.mean(dim=(2, 3), keepdim=True)
        g = F.silu(F.conv2d(g, sd[p + "channel_attention.1.weight"], sd[p + "channel_attention.1.bias"]))
        g = torch.sigmoid(F.conv2d(g, sd[p + "channel_attention.3.weight"], sd[p + "channel_attention.3.bias"]))
        y = y * g
    if cin == cout and stride == 1:                 # :73,131-132
        y = y + identity
    return y


def residual_mhc_layer(sd, p: str, x: Tensor, c: int, sk_iters: int) -> Tensor:
    """ResidualMHCLayer.forward, bottleneck branch (vision_backbone.py:160-196)."""
    y = conv_mhc_layer(sd, p + "blocks.0.", x, c, c // 2, 1, 1, sk_iters)
    y = conv_mhc_layer(sd, p + "blocks.1.", y, c // 2, c, 3, 1, sk_iters)
    y = conv_mhc_layer(sd, p + "projection.", y, c, c, 1, 1, sk_iters)
    return y + x


def backbone(sd, x: Tensor, cfg: OracleConfig) -> Dict[str, Tensor]:
    """HybridVisionBackbone.forward (vision_backbone.py:329-397), eval."""
    it = cfg.sk_iters
    bc = cfg.base_channels
    p = "backbone."
    x = conv_mhc_layer(sd, p + "stem.0.", x, 3, bc, 3, 2, it)
    x = conv_mhc_layer(sd, p + "stem.1.", x, bc, bc, 3, 1, it)
    x = conv_mhc_layer(sd, p + "stem.2.", x, bc, 2 * bc, 3, 1, it)
    x = F.max_pool2d(x, 2, 2)
    raw = {"stem": x}
    ch = [2 * bc, 4 * bc, 8 * bc, 16 * bc]
    cur = 2 * bc
    for i, (nb, co) in enumerate(zip(cfg.num_blocks, ch)):
        sp = f"{p}stages.{i}."
        x = conv_mhc_layer(sd, sp + "0.", x, cur, co, 3, 2 if i > 0 else 1, it)
        for j in range(1, nb):
            x = residual_mhc_layer(sd, f"{sp}{j}.", x, co, it)
        raw[f"stage_{i + 1}"] = x
        cur = co
    out = {
        "scale_small": mhc_nchw(sd, p + "enhance_small.", raw["stage_2"], it),
        "scale_medium": mhc_nchw(sd, p + "enhance_medium.", raw["stage_3"], it),
        "scale_large": mhc_nchw(sd, p + "enhance_large.", raw["stage_4"], it),
        "raw_features": raw,
    }
    return out


# ----------------------------------------------------------------------------------------
# a5/a6/a10-a13: transformer encoder (vit_encoder_decoder.py, manifold_layers.py:386-434)
# ----------------------------------------------------------------------------------------
def interp_positions(pe: Tensor, n: int) -> Tensor:
    """Linear interpolation of a [1, L, D] table to n positions (vit_encoder_decoder.py:490-499)."""
    return F.interpolate(pe.transpose(1, 2), size=(n,), mode="linear").transpose(1, 2)


def attention(sd, p: str, x: Tensor, it: int, heads: int = 8) -> Tensor:
    """MultiHeadManifoldAttention.forward (manifold_layers.py:386-434), eval, self-attention."""
    return attention_general(sd, p, x, x, x, it, heads)[0]


def attention_general(sd, p: str, query: Tensor, key: Tensor, value: Tensor, it: int, heads: int = 8,
                      key_padding_mask: Optional[Tensor] = None):
    """MultiHeadManifoldAttention.forward (manifold_layers.py:386-434), eval: q/k/v mHC
    projections (:400-402), scores * head_dim^-0.5 (:410), key_padding_mask filled with -inf
    (:413-417), softmax (:420), PV, out_proj (:430).  Returns (out, attn_weights)."""
    B, Lq, D = query.shape
    hd = D // heads
    q = mhc(sd, p + "q_proj.", query, it).reshape(B, Lq, heads, hd).transpose(1, 2)
    k = mhc(sd, p + "k_proj.", key, it).reshape(B, -1, heads, hd).transpose(1, 2)
    v = mhc(sd, p + "v_proj.", value, it).reshape(B, -1, heads, hd).transpose(1, 2)
    s = (q @ k.transpose(-2, -1)) * hd ** -0.5
    if key_padding_mask is not None:
        s = s.masked_fill(key_padding_mask.unsqueeze(1).unsqueeze(2), float("-inf"))
    w = torch.softmax(s, dim=-1)
    o = (w @ v).transpose(1, 2).reshape(B, Lq, D)
    return mhc(sd, p + "out_proj.", o, it), w


def encoder_block(sd, p: str, x: Tensor, it: int) -> Tensor:
    """TransformerEncoderBlock.forward (vit_encoder_decoder.py:174-210), eval."""
    a = attention(sd, p + "attention.", rmsnorm(x, sd[p + "norm1.scale"]), it)
    x = x + mhc(sd, p + "residual_mhc1.", a, it)
    h = rmsnorm(x, sd[p + "norm2.scale"])
    h = F.linear(F.gelu(F.linear(h, sd[p + "mlp.0.weight"], sd[p + "mlp.0.bias"])),
                 sd[p + "mlp.3.weight"], sd[p + "mlp.3.bias"])
    return x + mhc(sd, p + "residual_mhc2.", h, it)


def vit_encoder(sd, x: Tensor, cfg: OracleConfig) -> Tensor:
    """VisionTransformerEncoder.forward (vit_encoder_decoder.py:277-315) -> CLS [B, D].

    PatchEmbedding (:77-108) with shim S3: the 256 learned patch positions are linearly
    interpolated to H*W (CLS slot kept) when the grid is not 16x16.
    """
    it = cfg.sk_iters
    p = "vit_encoder.vit_encoder."
    B = x.shape[0]
    t = F.conv2d(x, sd[p + "patch_embed.projection.weight"], sd[p + "patch_embed.projection.bias"])
    t = t.flatten(2).transpose(1, 2)                                   # [B, N, D]
    t = mhc(sd, p + "patch_embed.mhc_enhance.", t, it)
    cls = sd[p + "patch_embed.cls_token"].expand(B, -1, -1)
    t = torch.cat([cls, t], dim=1)
    pe = sd[p + "patch_embed.position_embeddings"]
    if pe.shape[1] != t.shape[1]:
        pe = torch.cat([pe[:, :1], interp_positions(pe[:, 1:], t.shape[1] - 1)], dim=1)
    t = rmsnorm(t + pe, sd[p + "patch_embed.norm.scale"])
    for i in range(cfg.vit_depth):
        t = encoder_block(sd, f"{p}blocks.{i}.", t, it)
    t = rmsnorm(t, sd[p + "norm.scale"])
    return t[:, 0]


def hybrid_encoder(sd, cnn: Tensor, cfg: OracleConfig) -> Tensor:
    """HybridVisionEncoder.forward (vit_encoder_decoder.py:470-520) with shim S2 on fusion_mhc."""
    p = "vit_encoder."
    B, C, H, W = cnn.shape
    v = F.conv2d(cnn, sd[p + "cnn_to_vit.weight"], sd[p + "cnn_to_vit.bias"])
    v = v.flatten(2).transpose(1, 2)
    pe = sd[p + "pos_embed"]
    v = v + (pe if H * W == pe.shape[1] else interp_positions(pe, H * W))
    v = v.reshape(B, H, W, -1).permute(0, 3, 1, 2)
    cls = vit_encoder(sd, v, cfg)                                      # [B, 256]
    g = cls[:, :, None, None].expand(-1, -1, H, W)
    e = F.conv2d(g, sd[p + "vit_to_cnn.weight"], sd[p + "vit_to_cnn.bias"])
    return mhc_nchw(sd, p + "fusion_mhc.", cnn + e, cfg.sk_iters)


# ----------------------------------------------------------------------------------------
# a14: FPN (feature_fusion.py:82-153) with shim S2
# ----------------------------------------------------------------------------------------
def fpn(sd, feats: Dict[str, Tensor], cfg: OracleConfig) -> Dict[str, Tensor]:
    p = "feature_fusion."
    it = cfg.sk_iters

    def lateral(i, x):
        return F.conv2d(x, sd[f"{p}lateral_convs.{i}.weight"], sd[f"{p}lateral_convs.{i}.bias"])

    def refine(i, x):
        q = f"{p}refinement_convs.{i}."
        x = F.relu(batchnorm_eval(F.conv2d(x, sd[q + "0.weight"], sd[q + "0.bias"], 1, 1), sd, q + "1."))
        x = F.relu(batchnorm_eval(F.conv2d(x, sd[q + "3.weight"], sd[q + "3.bias"], 1, 1), sd, q + "4."))
        return mhc_nchw(sd, f"{p}mhc_fusions.{i}.", x, it)

    def out(i, x):
        return F.conv2d(x, sd[f"{p}output_convs.{i}.weight"], sd[f"{p}output_convs.{i}.bias"])

    pl = lateral(2, feats["scale_large"])
    pm = lateral(1, feats["scale_medium"])
    ps = lateral(0, feats["scale_small"])
    rl = refine(2, pl)
    res = {"fused_large": out(2, rl)}
    rm = refine(1, pm + F.interpolate(rl, size=pm.shape[2:], mode="nearest"))
    res["fused_medium"] = out(1, rm)
    rs = refine(0, ps + F.interpolate(rm, size=ps.shape[2:], mode="nearest"))
    res["fused_small"] = out(0, rs)
    return res


# ----------------------------------------------------------------------------------------
# a15-a17: YOLO head + decoder (yolo_head.py) with shims S4/S5
# ----------------------------------------------------------------------------------------
def prediction_head(sd, p: str, x: Tensor, it: int, num_classes: int, A: int = 3) -> Tensor:
    """YOLOPredictionHead.forward (yolo_head.py:170-203) -> [B, A, H, W, 5+C]."""
    x = F.leaky_relu(batchnorm_eval(F.conv2d(x, sd[p + "conv_layers.0.weight"], sd[p + "conv_layers.0.bias"], 1, 1),
                                    sd, p + "conv_layers.1."), 0.1)
    x = F.leaky_relu(batchnorm_eval(F.conv2d(x, sd[p + "conv_layers.3.weight"], sd[p + "conv_layers.3.bias"], 1, 1),
                                    sd, p + "conv_layers.4."), 0.1)
    x = mhc_nchw(sd, p + "mhc_enhance.", x, it)
    y = F.conv2d(x, sd[p + "pred_conv.weight"], sd[p + "pred_conv.bias"])
    B, _, H, W = y.shape
    return y.view(B, A, 5 + num_classes, H, W).permute(0, 1, 3, 4, 2)


def anchor_wh(scale: int, anchors=None) -> Tensor:
    """Per-scale anchor w,h normalised by 416 (yolo_head.py:27-31,48-51; shim S4)."""
    a = (anchors or DEFAULT_ANCHORS)[scale]
    return torch.tensor([[w / 416.0, h / 416.0] for (w, h) in a], dtype=torch.float64)


def decode(pred: Tensor, awh: Tensor) -> Dict[str, Tensor]:
    """YOLODecoder.forward (yolo_head.py:220-294) with shim S5 (boxes [B,A,H,W,4])."""
    B, A, H, W, _ = pred.shape
    xy = torch.sigmoid(pred[..., 0:2])
    wh = pred[..., 2:4]
    obj = torch.sigmoid(pred[..., 4:5])
    cls = torch.sigmoid(pred[..., 5:])
    gy, gx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    gx = gx.view(1, 1, H, W).to(pred.dtype)
    gy = gy.view(1, 1, H, W).to(pred.dtype)
    bx = (gx + xy[..., 0]) / W
    by = (gy + xy[..., 1]) / H
    aw = awh[:, 0].to(pred.dtype).view(1, A, 1, 1)
    ah = awh[:, 1].to(pred.dtype).view(1, A, 1, 1)
    bw = aw * torch.exp(wh[..., 0])
    bh = ah * torch.exp(wh[..., 1])
    boxes = torch.stack([bx - bw / 2, by - bh / 2, bx + bw / 2, by + bh / 2], dim=-1)
    scores = obj * cls
    cs, ci = torch.max(scores, dim=-1)
    return {"boxes": boxes, "scores": scores, "class_scores": cs, "class_indices": ci,
            "objectness": obj, "raw_predictions": pred}


# ----------------------------------------------------------------------------------------
# a18: system forward (hybrid_vision.py:222-402) with shim S6
# ----------------------------------------------------------------------------------------
def final_features(sd, fused: Dict[str, Tensor], cfg: OracleConfig) -> Tensor:
    """_extract_final_features (hybrid_vision.py:369-402): GAP x3 -> cat -> mHC -> Linear/ReLU/Linear."""
    pooled = [fused[k].mean(dim=(2, 3)) for k in ("fused_small", "fused_medium", "fused_large")]
    c = mhc(sd, "final_fusion.", torch.cat(pooled, dim=1), cfg.sk_iters)
    c = F.relu(F.linear(c, sd["output_projection.2.weight"], sd["output_projection.2.bias"]))
    return F.linear(c, sd["output_projection.4.weight"], sd["output_projection.4.bias"])


def system_forward(sd: Dict[str, Tensor], x: Tensor, cfg: OracleConfig = BASE) -> Dict:
    """HybridVisionSystem.forward(x, task='detection') in eval mode."""
    bb = backbone(sd, x, cfg)
    vit = hybrid_encoder(sd, bb["scale_large"], cfg)
    bb["scale_large"] = (bb["scale_large"] + vit) / 2
    fused = fpn(sd, bb, cfg)
    det_in = {"scale_small": fused["fused_small"], "scale_medium": fused["fused_medium"],
              "scale_large": fused["fused_large"]}
    preds, decoded = {}, {}
    for s, key in enumerate(("scale_small", "scale_medium", "scale_large")):
        pr = prediction_head(sd, f"detection_head.pred_heads.{s}.", det_in[key], cfg.sk_iters, cfg.num_classes)
        preds[f"scale_{s}"] = pr
        decoded[f"scale_{s}"] = decode(pr, anchor_wh(s))
    return {"backbone_features": bb, "vit_features": vit, "fused_features": fused,
            "predictions": preds, "decoded": decoded,
            "final_features": final_features(sd, fused, cfg)}


def cast_state_dict(sd: Dict[str, Tensor], dtype=torch.float32) -> Dict[str, Tensor]:
    return {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}


# ----------------------------------------------------------------------------------------
# §8f-1: detection post-processing (yolo_head.py:571-731)
# ----------------------------------------------------------------------------------------
def _iou(b1: Tensor, b2: Tensor) -> Tensor:
    """compute_iou (yolo_head.py:733-756)."""
    ix1 = torch.max(b1[..., 0], b2[..., 0])
    iy1 = torch.max(b1[..., 1], b2[..., 1])
    ix2 = torch.min(b1[..., 2], b2[..., 2])
    iy2 = torch.min(b1[..., 3], b2[..., 3])
    inter = (ix2 - ix1).clamp(min=0) * (iy2 - iy1).clamp(min=0)
    a1 = (b1[..., 2] - b1[..., 0]) * (b1[..., 3] - b1[..., 1])
    a2 = (b2[..., 2] - b2[..., 0]) * (b2[..., 3] - b2[..., 1])
    return inter / (a1 + a2 - inter + 1e-6)


def nms(boxes: Tensor, scores: Tensor, iou_thr: float, max_det: int) -> List[int]:
    """non_max_suppression (yolo_head.py:678-731): greedy, best first, keep IoU < thr.  The sort
    is the reference's own call (yolo_head.py:700): torch.sort's default, NOT stable -- on the CPU
    libstdc++ introsort, whose tie order oracle/std_sort.py restates."""
    order = torch.sort(scores, descending=True).indices
    keep: List[int] = []
    while order.numel() > 0:
        i = int(order[0])
        keep.append(i)
        if len(keep) >= max_det:
            break
        rest = order[1:]
        if rest.numel() == 0:
            break
        order = rest[_iou(boxes[i].unsqueeze(0), boxes[rest]) < iou_thr]
    return keep


def post_process(decoded: Dict, conf_thr: float = 0.5, iou_thr: float = 0.5, max_det: int = 100):
    """YOLODetectionHead.post_process (yolo_head.py:571-676): per scale threshold + NMS,
    then NMS over the concatenation of the per-scale survivors."""
    per_scale = []
    B = None
    for key in sorted(decoded):
        out = decoded[key]
        scores = out["class_scores"]
        B = scores.shape[0]
        bf, sf, cf = out["boxes"].reshape(B, -1, 4), scores.reshape(B, -1), out["class_indices"].reshape(B, -1)
        dets = []
        for b in range(B):
            m = sf[b] > conf_thr
            bb, ss, cc = bf[b][m], sf[b][m], cf[b][m]
            k = nms(bb, ss, iou_thr, max_det) if bb.numel() else []
            dets.append((bb[k], ss[k], cc[k]))
        per_scale.append(dets)
    res = []
    for b in range(B):
        ab = torch.cat([d[b][0].reshape(-1, 4) for d in per_scale])
        asc = torch.cat([d[b][1] for d in per_scale])
        al = torch.cat([d[b][2] for d in per_scale])
        k = nms(ab, asc, iou_thr, max_det) if ab.numel() else []
        res.append({"boxes": ab[k], "scores": asc[k], "labels": al[k]})
    return res
