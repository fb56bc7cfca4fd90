"""Autograd Functions of the training step over the HIP kernels.

Each Function's forward and backward launch hand-written gfx950 kernels through ops /
ops_train; torch only does the autograd bookkeeping (and a handful of parameter-sized fp32
glue ops in the mHC coefficient backward).  Activations are token-major NHWC / [T, D] in
the compute dtype; parameter gradients are fp32.

Dropout masks are never stored: forward and backward regenerate keep(seed, element) in the
kernels (hv_common.h hv_drop_scale); seeds come from ``next_seed`` (a host counter seeded
from torch's CPU generator, so runs are reproducible under torch.manual_seed).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from . import ops
from . import ops_train as T
from .ops import f32

Tensor = torch.Tensor


def next_seed() -> int:
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


def _need(ctx, i: int) -> bool:
    return bool(ctx.needs_input_grad[i])


# =============================================================================== conv
class ConvFn(torch.autograd.Function):
    """Conv2d (+ bias) on NHWC, optionally followed by training BatchNorm + activation
    (vision_backbone.py:42-49,113; feature_fusion.py:33-49; yolo_head.py:120-139)."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, conv, bn, act: str):
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        dt = x.dtype
        w = ops.conv_weight_prep(weight, dt)
        pre = ops.conv2d(x, w, k, s, p, bias=f32(bias) if bias is not None else None,
                         act="none" if bn is not None else act)
        ctx.meta = (k, s, p, act, bn is not None, x.shape[1:3])
        if bn is not None:
            momentum = bn.momentum if bn.momentum is not None else 0.1
            mean, rstd = T.bn_stats(pre, bn.eps, momentum, bn.running_mean if bn.track_running_stats else None,
                                    bn.running_var if bn.track_running_stats else None)
            if bn.track_running_stats and bn.num_batches_tracked is not None:
                bn.num_batches_tracked.add_(1)
            y = T.bn_apply(pre, mean, rstd, gamma, beta, act)
            ctx.save_for_backward(x, weight, pre, mean, rstd, gamma, beta)
        else:
            y = pre
            ctx.save_for_backward(x, weight, pre if act != "none" else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        k, s, p, act, has_bn, in_hw = ctx.meta
        dy = dy.contiguous()
        dgamma = dbeta = None
        if has_bn:
            x, weight, pre, mean, rstd, gamma, beta = ctx.saved_tensors
            dpre, dgamma, dbeta = T.bn_backward(pre, dy, mean, rstd, gamma, beta, act)
        else:
            x, weight, pre = ctx.saved_tensors
            dpre = T.act_backward(dy, pre, act) if act != "none" else dy
        cout, cin = weight.shape[0], weight.shape[1]
        # the GEMM operands need 16-byte rows: pad an odd channel count (YOLO's 255) with zeros
        epc = 8 if dpre.dtype == torch.bfloat16 else 4
        cp = (cout + epc - 1) // epc * epc
        wpad = weight
        if cp != cout:
            dpre = torch.nn.functional.pad(dpre, (0, cp - cout)).contiguous()
            wpad = torch.cat([weight.detach(), weight.new_zeros((cp - cout,) + tuple(weight.shape[1:]))], 0)
        dx = dw = db = None
        if _need(ctx, 0):
            flip = s == 1
            wt = T.dgrad_weight(wpad, dpre.dtype, flip)
            dx = T.conv_dgrad(dpre, wt, k, s, p, in_hw, flipped=flip)
        if _need(ctx, 1):
            dst = T.grad_out(weight) if cp == cout else None
            dw = T.conv_grad_reorder(T.conv_wgrad(dpre, x, k, s, p), cp, cin, k, out=dst)[:cout]
        if _need(ctx, 2):
            db = T.colsum(dpre)[:cout]
        return dx, dw, db, dgamma, dbeta, None, None, None


def conv(x, conv, bn=None, act: str = "none"):
    return ConvFn.apply(x, conv.weight, conv.bias, bn.weight if bn is not None else None,
                        bn.bias if bn is not None else None, conv, bn, act)


# =============================================================================== linear
class LinearFn(torch.autograd.Function):
    """y = dropout(act(x W^T + b)) on [T, K] tokens (transformer MLP, output projection)."""

    @staticmethod
    def forward(ctx, x, weight, bias, act: str, p: float, seed: int, out_dtype):
        dt = x.dtype
        w = ops.cast(f32(weight), dt)
        if act == "none" and p == 0.0:
            y = ops.gemm(x, w, bias=f32(bias) if bias is not None else None, out_dtype=out_dtype)
            pre = None
        else:
            pre = torch.empty((x.shape[0], w.shape[0]), device=x.device, dtype=out_dtype or dt)
            y = T.gemm_train(x, w, mode=1, act=act, aux=pre, bias=f32(bias) if bias is not None else None,
                             drop_p=p, seed=seed, out_dtype=out_dtype)
        ctx.meta = (act, p, seed)
        ctx.save_for_backward(x, weight, pre)
        return y

    @staticmethod
    def backward(ctx, dy):
        act, p, seed = ctx.meta
        x, weight, pre = ctx.saved_tensors
        dy = dy.contiguous()
        dt = x.dtype
        if pre is not None:
            g = T.act_backward(dy.to(pre.dtype), pre, act, p, seed)
        else:
            g = dy
        g = g.to(dt) if g.dtype != dt else g
        dx = dw = db = None
        if _need(ctx, 0):
            dx = ops.gemm(g, T.transpose_cast(weight, dt))
        if _need(ctx, 1):
            dw = T.wgrad(g, x, out=T.grad_out(weight))
        if _need(ctx, 2):
            db = T.colsum(g)
        return dx, dw, db, None, None, None, None


def linear(x, lin, act="none", p=0.0, out_dtype=None):
    return LinearFn.apply(x, lin.weight, lin.bias, act, p, next_seed() if p > 0 else 0, out_dtype)


# =============================================================================== Sinkhorn
class SinkhornGroupFn(torch.autograd.Function):
    """All Sinkhorn projections of the model in one grouped forward / backward
    (manifold_layers.py:32-93 and its autograd)."""

    @staticmethod
    def forward(ctx, group, token, *raws):
        outs = group.run(list(raws))
        ctx.group = group
        ctx.token = token                  # train_model._InFlight: the group's buffers are in use
        ctx.set_materialize_grads(False)
        return tuple(o.squeeze(0) if r.dim() == 2 else o for o, r in zip(outs, raws))

    @staticmethod
    def backward(ctx, *douts):
        g = ctx.group
        draws = g.backward(list(douts))
        if ctx.token is not None:          # the Sinkhorn backward runs after every mHC backward
            ctx.token.release()
        # a projection no loss depends on gets no gradient at all (None, as the reference's
        # per-module autograd leaves it): the optimizer then skips that H_res_raw
        return (None, None) + tuple(d if o is not None else None for d, o in zip(draws, douts))


# =============================================================================== mHC
def _mhc_coefficients(m, H_res: Tensor, W1: Tensor, b1: Tensor, dt):
    """Folded coefficients in fp32 + the compute-dtype GEMM operands."""
    gc, u, wct = ops.mhc_prep(m.H_pre_raw, m.H_post_raw, H_res, m.norm_pre.weight, m.norm_pre.bias,
                              gc_transposed=False)
    w1 = f32(W1)
    if dt == torch.bfloat16:                       # [D, 2Hd] = Gc W1^T on the bf16 MFMA (fp32 result)
        A1 = ops.gemm(ops.cast(gc, dt), ops.cast(w1, dt), out_dtype=torch.float32)
    else:
        A1 = ops.gemm(gc, w1)
    c1 = ops.gemv(w1, u, b1)                       # [2Hd]
    return gc, u, wct, A1, c1


EPILOGUE_COLSUM = True    # mHC bias gradients from the dgrad GEMM epilogue (tools/train_ab.py TF.EPILOGUE_COLSUM)


class MhcFn(torch.autograd.Function):
    """ManifoldHyperConnection.forward in training mode (manifold_layers.py:223-280):
    LN_pre -> (H_pre . Linear1 folded) -> GELU -> dropout -> Linear2 -> GELU -> dropout ->
    [x | h2] Wc -> LN_post -> dropout, with the full backward (incl. constrained-matrix
    gradients down to H_pre_raw / H_post_raw / H_res)."""

    @staticmethod
    def forward(ctx, x, H_res, H_pre_raw, H_post_raw, g_pre, b_pre, W1, b1, W2, b2, g_post, b_post, m, seeds,
                coef=None, out_f32=False):
        dt = x.dtype
        D, Hd = m.input_dim, m.hidden_dim
        p1, p2, p3 = m.mlp[2].p, m.mlp[5].p, m.dropout.p
        s1, s2, s3 = seeds
        with torch.no_grad():
            if coef is not None:                            # grouped prep of the whole model (train_prep)
                gc = u = wct = A1 = None
                a1t, c1, w2, wct_dt = coef.a1t, coef.c1, coef.w2, coef.wct
                ctx.coef, ctx.coef_gen = coef, coef.gen
            else:
                gc, u, wct, A1, c1 = _mhc_coefficients(m, H_res, W1, b1, dt)
                a1t = T.transpose_cast(A1, dt)              # [2Hd, D]
                w2 = ops.cast(f32(W2), dt)
                wct_dt = ops.cast(wct, dt)                  # [D, D+Hd]
                ctx.coef = None
            z, mean, rstd = T.rownorm_train(T.LN, x, 1e-5)
            pre1 = torch.empty((x.shape[0], 2 * Hd), device=x.device, dtype=dt)
            h1 = T.gemm_train(z, a1t, mode=1, act="gelu", aux=pre1, bias=c1, drop_p=p1, seed=s1)
            pre2 = torch.empty((x.shape[0], Hd), device=x.device, dtype=dt)
            h2 = T.gemm_train(h1, w2, mode=1, act="gelu", aux=pre2, bias=f32(b2), drop_p=p2, seed=s2)
            yc = ops.gemm(x, wct_dt, a2=h2, out_dtype=torch.float32)
            # out_f32: the output in fp32 (autocast's LayerNorm output dtype, manifold_layers.py:248-270)
            # for sites that feed an fp32 residual stream (the ViT blocks' residual_mhc1/2)
            y, mean2, rstd2 = T.rownorm_train(T.LN, yc, 1e-5, g_post, b_post, p3, s3,
                                              out_dtype=torch.float32 if out_f32 else dt)
        ctx.m = m
        ctx.meta = (p1, p2, p3, s1, s2, s3)
        ctx.save_for_backward(x, z, mean, rstd, pre1, h1, pre2, h2, yc, mean2, rstd2, gc, u, wct, A1,
                              H_pre_raw, H_post_raw, g_pre, b_pre, W1, W2, g_post)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x, z, mean, rstd, pre1, h1, pre2, h2, yc, mean2, rstd2, gc, u, wct, A1,
         H_pre_raw, H_post_raw, g_pre, b_pre, W1, W2, g_post) = ctx.saved_tensors
        p1, p2, p3, s1, s2, s3 = ctx.meta
        m = ctx.m
        D, Hd = m.input_dim, m.hidden_dim
        dt = x.dtype
        dy = dy.contiguous()
        # LN_post (+ output dropout)
        co = ctx.coef
        if co is not None and co.gen != ctx.coef_gen:
            raise RuntimeError("MhcFn.backward: the grouped training coefficients were recomputed by a later "
                               "forward before this backward (one forward per backward)")
        dyc, dg_post, db_post = T.rownorm_backward(T.LN, yc, dy, mean2, rstd2, g_post, p3, s3, dx_dtype=dt)
        wc = co.wc if co is not None else T.transpose_cast(wct, dt)     # [D+Hd, D] (rows = input index)
        dwc_x = T.wgrad(x, dyc)                            # [D, D]
        dwc_h = T.wgrad(h2, dyc)                           # [Hd, D]
        dx_res = ops.gemm(dyc, wc[:D])                     # [T, D]
        # the bias gradients db2 / dc1 are summed in the dgrad GEMMs' epilogues (colsum=; the
        # separate column-sum pass over dpre when EPILOGUE_COLSUM is off)
        ecs = EPILOGUE_COLSUM
        db2 = torch.empty(Hd, device=x.device, dtype=torch.float32) if ecs else None
        dpre2 = T.gemm_train(dyc, wc[D:], mode=2, act="gelu", aux=pre2, drop_p=p2, seed=s2, colsum=db2)
        db2 = db2 if ecs else T.colsum(dpre2)
        dW2 = T.wgrad(dpre2, h1, out=T.grad_out(W2))       # [Hd, 2Hd]
        w2t = co.w2t if co is not None else T.transpose_cast(W2, dt)    # [2Hd, Hd]
        dc1 = torch.empty(2 * Hd, device=x.device, dtype=torch.float32) if ecs else None
        dpre1 = T.gemm_train(dpre2, w2t, mode=2, act="gelu", aux=pre1, drop_p=p1, seed=s1, colsum=dc1)
        dc1 = dc1 if ecs else T.colsum(dpre1)
        dA1t = T.wgrad(dpre1, z)                           # [2Hd, D]
        dz = ops.gemm(dpre1, co.a1 if co is not None else ops.cast(A1, dt))   # [T, D]
        dx, _, _ = T.rownorm_backward(T.LN, x, dz, mean, rstd, None, dx_dtype=dt, dx_add=dx_res,
                                      param_grads=False)
        # ---- coefficient backward (parameter-sized fp32)
        w1 = f32(W1)
        pdt = torch.bfloat16 if dt == torch.bfloat16 else torch.float32   # parameter-side GEMM operands
        if co is not None:
            gct, w1t, u = co.gct, co.w1t, co.u
        else:
            gct, w1t = T.transpose_cast(gc, pdt), T.transpose_cast(w1, torch.float32)
        dW1 = ops.gemm(ops.cast(dA1t, pdt), gct, out_dtype=torch.float32)  # dA1t Gc
        dW1 += torch.outer(dc1, u)
        db1 = dc1
        dGc = T.wgrad(dA1t, w1)                            # [D, Hd] = dA1t^T W1
        du = ops.gemv(w1t, dc1)                            # [Hd] = W1^T dc1 (hv_gemv)
        dH_pre_raw, dg_pre, db_pre, dH_res, dH_post_raw = T.mhc_param_backward(
            dGc, du, H_pre_raw, g_pre, b_pre, dwc_x, dwc_h, H_post_raw)
        return (dx, dH_res, dH_pre_raw, dH_post_raw, dg_pre, db_pre, dW1, db1, dW2, db2, dg_post, db_post,
                None, None, None, None)


def mhc(m, x: Tensor, H_res: Tensor, coef=None, out_f32: bool = False) -> Tensor:
    """coef: the site's train_prep.TrainCoef when the model's coefficients were prepared in one
    grouped pass (train_model.system_forward), else None (per-site preparation).  out_f32: fp32
    output whatever the compute dtype (autocast's LayerNorm output dtype)."""
    seeds = tuple(next_seed() if pp > 0 else 0 for pp in (m.mlp[2].p, m.mlp[5].p, m.dropout.p))
    y = MhcFn.apply(x, H_res, m.H_pre_raw, m.H_post_raw, m.norm_pre.weight, m.norm_pre.bias,
                    m.mlp[0].weight, m.mlp[0].bias, m.mlp[3].weight, m.mlp[3].bias,
                    m.norm_post.weight, m.norm_post.bias, m, seeds, coef, bool(out_f32))
    if m.training:                                   # a4: manifold_layers.py:275-276 (throttled)
        cnt = getattr(m, "_mon_count", 0)
        m._mon_count = cnt + 1
        every = getattr(m, "monitor_every", 1)
        if every > 0 and cnt % every == 0:
            m.monitor_stability(H_res, x, y)
    return y


# =============================================================================== SE gate
class SEGateFn(torch.autograd.Function):
    """y * sigmoid(W2 silu(W1 mean_hw(y) + b1) + b2) (+ identity)  (vision_backbone.py:76-85,126-132)."""

    @staticmethod
    def forward(ctx, y, identity, w1, b1, w2, b2):
        pooled = ops.channel_mean(y)
        gate = ops.se_mlp(pooled, w1.view(w1.shape[0], -1), b1, w2.view(w2.shape[0], -1), b2)
        out = ops.scale_residual(y, gate, identity)
        ctx.has_id = identity is not None
        ctx.save_for_backward(y, pooled, gate, w1, b1, w2, b2)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, pooled, gate, w1, b1, w2, b2 = ctx.saved_tensors
        dout = dout.contiguous()
        dgate = T.chan_dot(dout, y)
        dp, dw1, db1, dw2, db2 = T.se_mlp_backward(pooled, dgate, w1.view(w1.shape[0], -1), b1,
                                                   w2.view(w2.shape[0], -1), b2)
        dy = T.se_backward_apply(dout, gate, dp)
        did = dout if ctx.has_id else None
        return dy, did, dw1.view_as(w1), db1, dw2.view_as(w2), db2


# =============================================================================== elementwise
class AddFn(torch.autograd.Function):
    """(a + b) * alpha (hybrid_vision.py:256-258 and the residual adds)."""

    @staticmethod
    def forward(ctx, a, b, alpha: float):
        ctx.alpha = alpha
        return ops.add_scaled(a.contiguous(), b.contiguous(), alpha)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        if ctx.alpha == 1.0:
            return g, g, None
        s = T.dropout(g, 0.0, 0)
        s = ops.add_scaled(s, torch.zeros_like(s), ctx.alpha)
        return s, s, None


class DropAddFn(torch.autograd.Function):
    """res + dropout(x)  (vit_encoder_decoder.py:196,209: x = residual + dropout(mhc_out))."""

    @staticmethod
    def forward(ctx, res, x, p: float, seed: int):
        ctx.meta = (p, seed)
        d = T.dropout(x.contiguous(), p, seed) if p > 0 else x.contiguous()
        return ops.add_scaled(res.contiguous(), d, 1.0)

    @staticmethod
    def backward(ctx, g):
        p, seed = ctx.meta
        g = g.contiguous()
        return g, (T.dropout(g, p, seed) if p > 0 else g), None, None


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p: float, seed: int):
        ctx.meta = (p, seed)
        return T.dropout(x.contiguous(), p, seed)

    @staticmethod
    def backward(ctx, g):
        p, seed = ctx.meta
        return T.dropout(g.contiguous(), p, seed), None, None


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return ops.maxpool2x2(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return T.maxpool2x2_backward(x, g.contiguous())


class UpsampleAddFn(torch.autograd.Function):
    """a + nearest_upsample(b)  (feature_fusion.py:116-146)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.hw = b.shape[1:3]
        return ops.upsample_add(a.contiguous(), b.contiguous())

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        return g, T.upsample_backward(g, ctx.hw[0], ctx.hw[1])


class AddRowvecFn(torch.autograd.Function):
    """x[n, p, c] + v[n, c] (broadcast CLS projection, vit_encoder_decoder.py:505-512)."""

    @staticmethod
    def forward(ctx, x, v):
        return ops.add_rowvec(x.contiguous(), v)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        return g, T.chan_dot(g, None)


class RMSNormFn(torch.autograd.Function):
    """RMSNorm (manifold_layers.py:449-456)."""

    @staticmethod
    def forward(ctx, x, scale, eps: float, out_dtype=None):
        """out_dtype: the output dtype when it differs from x's (an fp32 residual stream normalised
        into a bf16 GEMM operand, or a bf16 tensor starting an fp32 stream)."""
        y, _, rstd = T.rownorm_train(T.RMS, x.contiguous(), eps, scale, out_dtype=out_dtype)
        ctx.save_for_backward(x, rstd, scale)
        return y

    @staticmethod
    def backward(ctx, g):
        x, rstd, scale = ctx.saved_tensors
        dx, dscale, _ = T.rownorm_backward(T.RMS, x.contiguous(), g.contiguous(), None, rstd, scale,
                                           dx_dtype=x.dtype)
        return dx, dscale, None, None


class GatherRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stride: int):
        ctx.stride = stride
        return ops.gather_rows(x.contiguous(), stride)

    @staticmethod
    def backward(ctx, g):
        return T.scatter_rows(g.contiguous(), ctx.stride), None


class VitAssembleFn(torch.autograd.Function):
    """cat(CLS, tokens) + positions (vit_encoder_decoder.py:100-106, before the RMSNorm)."""

    @staticmethod
    def forward(ctx, x, cls, pos):
        ctx.shapes = (cls.shape, pos.shape)
        return T.vit_assemble(x.contiguous(), cls.reshape(-1), pos)

    @staticmethod
    def backward(ctx, g):
        dx, dcls, dpos = T.vit_assemble_backward(g.contiguous())
        return dx, dcls.view(ctx.shapes[0]), dpos.view(ctx.shapes[1])


class CastFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.dt = x.dtype
        return x.to(dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dt), None


# =============================================================================== attention
class AttentionFn(torch.autograd.Function):
    """softmax(q k^T / sqrt(hd)) with dropout on the probabilities, times v
    (manifold_layers.py:404-427)."""

    @staticmethod
    def forward(ctx, q, k, v, heads: int, p: float, seed: int):
        o, lse = T.attention_train(q.contiguous(), k.contiguous(), v.contiguous(), heads, p, seed)
        ctx.meta = (heads, p, seed)
        ctx.save_for_backward(q, k, v, o, lse)
        return o

    @staticmethod
    def backward(ctx, g):
        heads, p, seed = ctx.meta
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = T.attention_backward(q, k, v, o, g.contiguous(), lse, heads, p, seed)
        return dq, dk, dv, None, None, None


# =============================================================================== loss
class YoloLossFn(torch.autograd.Function):
    """YOLOLoss of one scale (yolo_head.py:374-465): returns the scale's total_loss
    contribution (0-d) and the raw component sums [coord, obj, noobj, cls, total, n_obj]."""

    @staticmethod
    def forward(ctx, logits, targets, A: int, lambdas):
        sums, dl = T.yolo_loss(logits, targets, A, lambdas)
        ctx.save_for_backward(dl)
        ctx.mark_non_differentiable(sums)
        return sums[4].clone(), sums

    @staticmethod
    def backward(ctx, g, _gs):
        (dl,) = ctx.saved_tensors
        return dl * g.to(dl.dtype), None, None, None


from .runtime import carry_train_state  # noqa: E402

carry_train_state(globals())
