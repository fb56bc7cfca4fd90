"""Shared helpers for the NHWC conv path: per-forward parameter preparation and layout views."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import ops
from .runtime import RunCtx, current, module_options, resolve_dtype


def conv_prep(conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d], dtype: torch.dtype, owner: nn.Module):
    """(weight [cout, k*k*cin], scale[cout], bias[cout]) with eval-BN folded; cached per forward."""
    ctx = current()
    key = ("conv", id(conv))
    if ctx is not None and key in ctx.plans:
        return ctx.plans[key]
    cout = conv.out_channels
    dev = conv.weight.device
    if bn is not None and bn.training:
        raise RuntimeError("conv_prep folds eval-mode BatchNorm; training-mode BN (batch statistics) runs "
                           "through hv_amd.train_model -- call the module in train() mode instead")
    if ctx is not None and ctx.program is not None and ctx.program.dtype == dtype:
        ctx.program.add_conv(conv, bn)            # grouped from the next forward on
    if bn is not None:
        scale, bias = ops.bn_fold(cout, dev, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                  conv.bias, bn.eps)
    else:
        scale = None
        bias = ops.f32(conv.bias) if conv.bias is not None else None
    w = ops.conv_weight_prep(conv.weight, dtype)
    val = (w, scale, bias)
    if ctx is not None:
        ctx.plans[key] = val
    return val


def linear_prep(lin: nn.Linear, dtype: torch.dtype):
    ctx = current()
    key = ("linear", id(lin))
    if ctx is not None and key in ctx.plans:
        return ctx.plans[key]
    val = (ops.cast(ops.f32(lin.weight), dtype), ops.f32(lin.bias) if lin.bias is not None else None)
    if ctx is not None and ctx.program is not None and ctx.program.dtype == dtype:
        ctx.program.add_linear(lin)               # grouped from the next forward on
    if ctx is not None:
        ctx.plans[key] = val
    return val


def run_conv(x: torch.Tensor, conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d], act: str, owner: nn.Module,
             residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Conv2d(+BN eval)(+act) on NHWC x via the implicit-GEMM kernel."""
    dt = x.dtype
    w, s, b = conv_prep(conv, bn, dt, owner)
    k = conv.kernel_size[0]
    return ops.conv2d(x, w, k, conv.stride[0], conv.padding[0], scale=s, bias=b, act=act,
                      residual=residual)


def to_nchw_view(x: torch.Tensor) -> torch.Tensor:
    """NHWC storage -> NCHW-shaped (channels_last) view, zero-copy."""
    return x.permute(0, 3, 1, 2)


def to_nhwc(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """NCHW-shaped tensor -> contiguous NHWC in `dtype` (zero-copy for channels_last input)."""
    if x.dim() != 4:
        raise ValueError("expected a 4-D NCHW tensor")
    v = x.permute(0, 2, 3, 1)
    if v.is_contiguous() and v.dtype == dtype:
        return v
    if x.dtype == torch.float32 and x.is_contiguous():
        return ops.nchw_to_nhwc(x, dtype)
    return ops.nchw_to_nhwc(x.float().contiguous(), dtype)


class ctx_scope:
    """Enter a forward-scoped RunCtx unless one is already active."""

    def __init__(self, module: nn.Module):
        self.module = module
        self.own = None

    def __enter__(self) -> RunCtx:
        from .runtime import use_ctx
        c = current()
        if c is not None:
            return c
        self.own = use_ctx(RunCtx(dtype=resolve_dtype(self.module), opts=module_options(self.module)))
        return self.own.__enter__()

    def __exit__(self, *exc):
        if self.own is not None:
            self.own.__exit__(*exc)
        return False
