"""The C-ABI launchers as PyTorch dispatcher operators ``torch.ops.hv.*``.

Each op is a ``torch.library.custom_op`` over the same HIP launchers the modules call (ops.py /
ops_train.py), with
  * a fake (meta) kernel, so FakeTensor tracing -- ``torch.compile``, ``torch.export``, shape
    propagation -- sees the op and its output shapes without running the GPU code;
  * where the reference path is differentiable, autograd through the existing training
    Functions (train_fn.py): the backward re-runs that Function's forward on the saved inputs
    and differentiates it (recompute, nothing cached between the op's forward and backward).

The modules keep calling ops.* directly (no per-op dispatcher overhead on the ~1,250-launch
forward); these ops are the dispatcher-visible surface for user code, compilers and exporters.

Ops (reference function each replaces):
  hv::sinkhorn       SinkhornKnoppProjection.forward        manifold_layers.py:32-93
  hv::mhc            ManifoldHyperConnection.forward (eval)  manifold_layers.py:223-280
  hv::linear         nn.Linear + activation                  vit_encoder_decoder.py:146-152
  hv::conv_bn_act    Conv2d + eval BatchNorm + activation    vision_backbone.py:42-49,112-114
  hv::se_gate        SE gate (+ identity)                    vision_backbone.py:76-85,126-132
  hv::attention      softmax(QK^T/sqrt(hd)) V                manifold_layers.py:404-427
  hv::layernorm      nn.LayerNorm                            manifold_layers.py:250,267
  hv::rmsnorm        RMSNorm.forward                         manifold_layers.py:449-456
  hv::yolo_decode    YOLODecoder.forward (+S5)               yolo_head.py:220-294
  hv::nms            post_process + non_max_suppression      yolo_head.py:571-731
"""
from __future__ import annotations

import types
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import ops
from . import ops_train as T

_ACTS = ("none", "relu", "silu", "gelu", "leaky", "sigmoid")


def _grad_of(fn, inputs, grads_out):
    """Recompute fn(*inputs) with autograd on and return d(outputs . grads_out)/d(inputs)."""
    with torch.enable_grad():
        leaves = [t.detach().requires_grad_(t.is_floating_point()) if torch.is_tensor(t) else t for t in inputs]
        outs = fn(*leaves)
        outs = outs if isinstance(outs, (tuple, list)) else (outs,)
        pairs = [(o, g) for o, g in zip(outs, grads_out) if g is not None and o.requires_grad]
        want = [t for t in leaves if torch.is_tensor(t) and t.requires_grad]
        if not pairs or not want:
            return [None] * len(inputs)
        gs = torch.autograd.grad([o for o, _ in pairs], want, [g.contiguous() for _, g in pairs], allow_unused=True)
    it = iter(gs)
    return [next(it) if torch.is_tensor(t) and t.requires_grad else None for t in leaves]


# ----------------------------------------------------------------------------------- sinkhorn
@torch.library.custom_op("hv::sinkhorn", mutates_args=(), device_types="cuda")
def sinkhorn(raw: Tensor, iters: int, eps: float = 1e-8, tau: float = 1.0) -> Tuple[Tensor, Tensor]:
    M, hist = ops.sinkhorn(raw.float().contiguous(), iters, eps, tau)
    M = M.squeeze(0) if raw.dim() == 2 else M
    return M.clone(), hist[:iters].clone()


@sinkhorn.register_fake
def _(raw, iters, eps=1e-8, tau=1.0):
    return raw.new_empty(raw.shape, dtype=torch.float32), raw.new_empty((iters,), dtype=torch.float32)


def _sinkhorn_setup(ctx, inputs, output):
    raw, iters, eps, tau = inputs
    ctx.save_for_backward(raw)
    ctx.meta = (iters, eps, tau)


def _sinkhorn_bwd(ctx, dM, dhist):
    (raw,) = ctx.saved_tensors
    iters, eps, tau = ctx.meta
    g = ops.SinkhornGroup([raw.float().contiguous()], [iters], raw.device, eps, tau)
    g.run()
    (draw,) = g.backward([dM.reshape(g.outs[0].shape) if dM is not None else None])
    return draw.view(raw.shape), None, None, None


sinkhorn.register_autograd(_sinkhorn_bwd, setup_context=_sinkhorn_setup)


# ----------------------------------------------------------------------------------- mHC
def _mhc_namespace(H_pre_raw, H_post_raw, g_pre, b_pre, W1, b1, W2, b2, g_post, b_post):
    """The attribute view of a ManifoldHyperConnection that build_plan / MhcFn read."""
    D, Hd = H_pre_raw.shape
    lin = lambda w, b: types.SimpleNamespace(weight=w, bias=b)     # noqa: E731
    drop = types.SimpleNamespace(p=0.0)
    return types.SimpleNamespace(
        input_dim=D, hidden_dim=Hd, H_pre_raw=H_pre_raw, H_post_raw=H_post_raw,
        norm_pre=lin(g_pre, b_pre), norm_post=lin(g_post, b_post), dropout=drop, training=False,
        mlp=[lin(W1, b1), None, drop, lin(W2, b2), None, drop])


@torch.library.custom_op("hv::mhc", mutates_args=(), device_types="cuda")
def mhc(x: Tensor, H_pre_raw: Tensor, H_post_raw: Tensor, H_res_raw: Tensor, g_pre: Tensor, b_pre: Tensor,
        W1: Tensor, b1: Tensor, W2: Tensor, b2: Tensor, g_post: Tensor, b_post: Tensor,
        sk_iters: int = 20) -> Tensor:
    """x [T, D] (bf16 or fp32: the compute precision) -> LN_post(mHC(x)) [T, D], eval mode."""
    from .manifold import build_plan, mhc_apply
    m = _mhc_namespace(H_pre_raw, H_post_raw, g_pre, b_pre, W1, b1, W2, b2, g_post, b_post)
    h_res, _ = ops.sinkhorn(H_res_raw.float().contiguous(), sk_iters)
    return mhc_apply(x.contiguous(), build_plan(m, h_res.squeeze(0), x.dtype))


@mhc.register_fake
def _(x, H_pre_raw, H_post_raw, H_res_raw, g_pre, b_pre, W1, b1, W2, b2, g_post, b_post, sk_iters=20):
    return torch.empty_like(x)


def _mhc_train_graph(sk_iters):
    from .train_fn import MhcFn, SinkhornGroupFn

    def fn(x, H_pre_raw, H_post_raw, H_res_raw, g_pre, b_pre, W1, b1, W2, b2, g_post, b_post):
        g = ops.SinkhornGroup([H_res_raw.detach().float().contiguous()], [sk_iters], x.device)
        (h_res,) = SinkhornGroupFn.apply(g, None, H_res_raw)
        m = _mhc_namespace(H_pre_raw, H_post_raw, g_pre, b_pre, W1, b1, W2, b2, g_post, b_post)
        return MhcFn.apply(x, h_res, H_pre_raw, H_post_raw, g_pre, b_pre, W1, b1, W2, b2, g_post, b_post, m, (0, 0, 0))
    return fn


def _mhc_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs[:12])
    ctx.sk_iters = inputs[12]


def _mhc_bwd(ctx, dy):
    grads = _grad_of(_mhc_train_graph(ctx.sk_iters), list(ctx.saved_tensors), [dy])
    return tuple(grads) + (None,)


mhc.register_autograd(_mhc_bwd, setup_context=_mhc_setup)


# ----------------------------------------------------------------------------------- linear
@torch.library.custom_op("hv::linear", mutates_args=(), device_types="cuda")
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None, act: str = "none") -> Tensor:
    """act(x W^T + b) for x [T, K] in the compute dtype; fp32 weight [N, K]."""
    return ops.gemm(x.contiguous(), ops.cast(ops.f32(weight), x.dtype), bias=ops.f32(bias), act=act)


@linear.register_fake
def _(x, weight, bias=None, act="none"):
    return x.new_empty((x.shape[0], weight.shape[0]))


def _linear_setup(ctx, inputs, output):
    x, w, b, act = inputs
    ctx.save_for_backward(x, w, b)
    ctx.act = act


def _linear_bwd(ctx, dy):
    from .train_fn import LinearFn
    x, w, b = ctx.saved_tensors
    act = ctx.act
    dx, dw, db = _grad_of(lambda x_, w_, b_: LinearFn.apply(x_, w_, b_, act, 0.0, 0, None), [x, w, b], [dy])
    return dx, dw, db, None


linear.register_autograd(_linear_bwd, setup_context=_linear_setup)


# ----------------------------------------------------------------------------------- conv + BN
@torch.library.custom_op("hv::conv_bn_act", mutates_args=(), device_types="cuda")
def conv_bn_act(x: Tensor, weight: Tensor, bias: Optional[Tensor], bn_weight: Optional[Tensor],
                bn_bias: Optional[Tensor], bn_mean: Optional[Tensor], bn_var: Optional[Tensor],
                stride: int = 1, padding: int = 0, act: str = "none", eps: float = 1e-5) -> Tensor:
    """Implicit-GEMM conv of NHWC x [n, h, w, cin] (compute dtype) with eval BatchNorm folded
    into the epilogue, then the activation; weight [cout, cin, k, k] fp32.  Inference only
    (training-mode BN -- batch statistics, running-stat updates -- is the module path)."""
    k = weight.shape[-1]
    if bn_weight is not None:
        scale, b = ops.bn_fold(weight.shape[0], x.device, bn_weight, bn_bias, bn_mean, bn_var, bias, eps)
    else:
        scale, b = None, ops.f32(bias)
    w = ops.conv_weight_prep(weight, x.dtype, scale)
    return ops.conv2d(x.contiguous(), w, k, stride, padding, bias=b, act=act)


@conv_bn_act.register_fake
def _(x, weight, bias, bn_weight, bn_bias, bn_mean, bn_var, stride=1, padding=0, act="none", eps=1e-5):
    n, h, w, _ = x.shape
    k = weight.shape[-1]
    oh = (h + 2 * padding - k) // stride + 1
    ow = (w + 2 * padding - k) // stride + 1
    return x.new_empty((n, oh, ow, weight.shape[0]))


# ----------------------------------------------------------------------------------- SE gate
@torch.library.custom_op("hv::se_gate", mutates_args=(), device_types="cuda")
def se_gate(y: Tensor, identity: Optional[Tensor], w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor) -> Tensor:
    """y * sigmoid(W2 silu(W1 mean_hw(y) + b1) + b2) (+ identity); y NHWC."""
    gate = ops.se_gate(y.contiguous(), w1.reshape(w1.shape[0], -1), b1, w2.reshape(w2.shape[0], -1), b2)
    return ops.scale_residual(y.contiguous(), gate, None if identity is None else identity.contiguous())


@se_gate.register_fake
def _(y, identity, w1, b1, w2, b2):
    return torch.empty_like(y)


def _se_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _se_bwd(ctx, dout):
    from .train_fn import SEGateFn
    return tuple(_grad_of(SEGateFn.apply, list(ctx.saved_tensors), [dout]))


se_gate.register_autograd(_se_bwd, setup_context=_se_setup)


# ----------------------------------------------------------------------------------- attention
@torch.library.custom_op("hv::attention", mutates_args=(), device_types="cuda")
def attention(q: Tensor, k: Tensor, v: Tensor, heads: int) -> Tensor:
    """q, k, v [n, L, D] -> softmax(q k^T / sqrt(D / heads)) v per head."""
    return ops.attention(q.contiguous(), k.contiguous(), v.contiguous(), heads)


@attention.register_fake
def _(q, k, v, heads):
    return torch.empty_like(q)


def _attn_setup(ctx, inputs, output):
    q, k, v, heads = inputs
    ctx.save_for_backward(q, k, v)
    ctx.heads = heads


def _attn_bwd(ctx, do):
    from .train_fn import AttentionFn
    heads = ctx.heads
    g = _grad_of(lambda q, k, v: AttentionFn.apply(q, k, v, heads, 0.0, 0), list(ctx.saved_tensors), [do])
    return g[0], g[1], g[2], None


attention.register_autograd(_attn_bwd, setup_context=_attn_setup)


# ----------------------------------------------------------------------------------- norms
@torch.library.custom_op("hv::layernorm", mutates_args=(), device_types="cuda")
def layernorm(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], eps: float = 1e-5) -> Tensor:
    return ops.layernorm(x.contiguous(), ops.f32(weight), ops.f32(bias), eps)


@layernorm.register_fake
def _(x, weight, bias, eps=1e-5):
    return torch.empty_like(x)


def _ln_setup(ctx, inputs, output):
    x, w, b, eps = inputs
    ctx.save_for_backward(x, w, b)
    ctx.eps = eps


def _ln_bwd(ctx, dy):
    x, w, b = ctx.saved_tensors
    xc = x.contiguous()
    _, mean, rstd = T.rownorm_train(T.LN, xc, ctx.eps, w, b)
    dx, dw, db = T.rownorm_backward(T.LN, xc, dy.contiguous(), mean, rstd, w, dx_dtype=x.dtype,
                                    param_grads=w is not None)
    return dx, dw, db, None


layernorm.register_autograd(_ln_bwd, setup_context=_ln_setup)


@torch.library.custom_op("hv::rmsnorm", mutates_args=(), device_types="cuda")
def rmsnorm(x: Tensor, scale: Tensor, eps: float = 1e-8) -> Tensor:
    return ops.rmsnorm(x.contiguous(), ops.f32(scale), eps)


@rmsnorm.register_fake
def _(x, scale, eps=1e-8):
    return torch.empty_like(x)


def _rms_setup(ctx, inputs, output):
    x, s, eps = inputs
    ctx.save_for_backward(x, s)
    ctx.eps = eps


def _rms_bwd(ctx, dy):
    from .train_fn import RMSNormFn
    x, s = ctx.saved_tensors
    eps = ctx.eps
    shp = x.shape
    g = _grad_of(lambda x_, s_: RMSNormFn.apply(x_.reshape(-1, shp[-1]), s_, eps).view(shp), [x, s], [dy])
    return g[0], g[1], None


rmsnorm.register_autograd(_rms_bwd, setup_context=_rms_setup)


# ----------------------------------------------------------------------------------- detection
@torch.library.custom_op("hv::yolo_decode", mutates_args=(), device_types="cuda")
def yolo_decode(logits: Tensor, num_anchors: int, num_classes: int,
                anchor_wh: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """NHWC logits [n, h, w, A*(5+nc)] -> (predictions [n,A,h,w,5+nc], boxes xyxy, scores
    [.., nc], class_scores, class_indices (int64, first index on ties), objectness)."""
    d, _ = ops.yolo_decode(logits.contiguous(), num_anchors, num_classes, anchor_wh)
    return (d["raw_predictions"], d["boxes"], d["scores"], d["class_scores"], d["class_indices"], d["objectness"])


@yolo_decode.register_fake
def _(logits, num_anchors, num_classes, anchor_wh):
    n, h, w, _ = logits.shape
    A, P = num_anchors, 5 + num_classes
    f = lambda *s: logits.new_empty(s, dtype=torch.float32)     # noqa: E731
    return (f(n, A, h, w, P), f(n, A, h, w, 4), f(n, A, h, w, num_classes), f(n, A, h, w),
            logits.new_empty((n, A, h, w), dtype=torch.int64), f(n, A, h, w, 1))


@torch.library.custom_op("hv::nms", mutates_args=(), device_types="cuda")
def nms(boxes: List[Tensor], class_scores: List[Tensor], class_indices: List[Tensor], conf_threshold: float,
        iou_threshold: float, max_detections: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Per-scale decoded outputs -> (boxes [B, max_det, 4], scores [B, max_det], labels
    [B, max_det] int64, count [B] int32): post_process's per-scale threshold + greedy NMS, then
    the cross-scale NMS."""
    dec = {f"scale_{i}": {"boxes": b, "class_scores": s, "class_indices": c}
           for i, (b, s, c) in enumerate(zip(boxes, class_scores, class_indices))}
    return tuple(t.clone() for t in ops.nms_batched(dec, conf_threshold, iou_threshold, max_detections))


@nms.register_fake
def _(boxes, class_scores, class_indices, conf_threshold, iou_threshold, max_detections):
    B = boxes[0].shape[0]
    return (boxes[0].new_empty((B, max_detections, 4)), boxes[0].new_empty((B, max_detections)),
            boxes[0].new_empty((B, max_detections), dtype=torch.int64),
            boxes[0].new_empty((B,), dtype=torch.int32))


OPS = ("sinkhorn", "mhc", "linear", "conv_bn_act", "se_gate", "attention", "layernorm", "rmsnorm", "yolo_decode",
       "nms")
