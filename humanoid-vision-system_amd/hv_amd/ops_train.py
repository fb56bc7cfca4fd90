"""Torch-tensor wrappers over the training-step half of the libhvs C ABI.

Same rules as ops.py: every call launches HIP kernels on the current torch stream, writes
freshly allocated (caching-allocator) tensors, and there is no CPU fallback.  Parameter
gradients are fp32; activation gradients keep the activation dtype.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch
from torch.autograd.graph import increment_version

from . import _lib as L
from ._lib import check, dtype_code, ptr, stream_ptr
from .ops import _contig, _cuda, f32
from .runtime import options, seed_offset_ptr

Tensor = torch.Tensor


def _work(n: int, device) -> Tensor:
    return torch.empty(max(int(n), 1), device=device, dtype=torch.float32)


# ---------------------------------------------------------------------------- GEMMs
def gemm_train(a: Tensor, b: Tensor, *, mode: int, act: str = "none", aux: Optional[Tensor] = None,
               bias: Optional[Tensor] = None, drop_p: float = 0.0, seed: int = 0,
               residual: Optional[Tensor] = None, a_mean: Optional[Tensor] = None,
               a_rstd: Optional[Tensor] = None, b_colsum: Optional[Tensor] = None, a2: Optional[Tensor] = None,
               out_dtype: Optional[torch.dtype] = None, alpha: float = 1.0,
               colsum: Optional[Tensor] = None) -> Tensor:
    """C = A' B^T with a training epilogue (hv_gemm_desc.epi_mode):
    mode 1: aux <- pre-activation (written), C = dropout(act(pre));
    mode 2: C = acc * keep * act'(aux) (+ residual)  -- gradient through act + dropout.
    colsum (mode 2, fp32 [N]): receives the column sums of C as stored (the bias gradient of the
    layer), summed in the GEMM's epilogue (hv_gemm_desc.colsum_part) -- or, where the call takes
    another kernel, by a separate pass over C."""
    _cuda(a, b)
    M, K1 = a.shape
    K = K1 + (a2.shape[1] if a2 is not None else 0)
    N = b.shape[0]
    if b.shape[1] != K or a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError(f"gemm_train shape mismatch a {tuple(a.shape)} b {tuple(b.shape)}")
    od = out_dtype or a.dtype
    out = torch.empty((M, N), device=a.device, dtype=od)
    d = L.GemmDesc()
    d.dtype = dtype_code(a.dtype)
    d.M, d.N, d.K = M, N, K
    d.A, d.lda = a.data_ptr(), a.stride(0)
    if a2 is not None:
        d.A2, d.lda2, d.k1 = a2.data_ptr(), a2.stride(0), K1
    d.B, d.ldb = b.data_ptr(), b.stride(0)
    d.C, d.ldc, d.c_dtype = out.data_ptr(), N, dtype_code(od)
    d.a_mean, d.a_rstd = ptr(a_mean), ptr(a_rstd)
    d.b_colsum = ptr(b_colsum) if a_mean is not None else None
    d.bias = ptr(bias)
    d.act = L.ACT[act]
    d.alpha = alpha
    d.epi_mode = mode
    if mode:
        if aux is None or aux.shape != (M, N) or not aux.is_contiguous():
            raise ValueError("gemm_train: aux must be a contiguous [M, N] tensor")
        d.aux, d.ld_aux, d.aux_dtype = aux.data_ptr(), N, dtype_code(aux.dtype)
    d.drop_p, d.drop_seed = float(drop_p), int(seed) & 0xFFFFFFFF
    d.seed_offset = seed_offset_ptr()
    if residual is not None:
        _contig(residual, "residual")
        d.residual, d.ldr, d.r_dtype = residual.data_ptr(), N, dtype_code(residual.dtype)
    d.variant = options().gemm_variant
    what = f"hv_gemm(train mode {mode}) M={M} N={N} K={K}"
    if colsum is not None:
        if mode != 2 or colsum.shape != (N,) or colsum.dtype != torch.float32 or not colsum.is_contiguous():
            raise ValueError("gemm_train: colsum needs mode 2 and a contiguous fp32 [N] tensor")
        part = torch.empty((-(-M // 128) * 2) * N, device=a.device, dtype=torch.float32)
        d.colsum_part = part.data_ptr()
        rc = L.lib().hv_gemm(C.byref(d), stream_ptr())
        if rc != -2:                                  # HV_EUNSUPPORTED: nothing was launched
            check(rc, what)
            check(L.lib().hv_colsum_final(part.data_ptr(), -(-M // 64), N, colsum.data_ptr(), 0, stream_ptr()),
                  "hv_colsum_final")
            return out
        d.colsum_part = None
    check(L.lib().hv_gemm(C.byref(d), stream_ptr()), what)
    if colsum is not None:
        colsum.copy_(_colsum_pass(out))
    return out


def conv_dgrad(dy: Tensor, wt: Tensor, k: int, stride: int, pad: int, in_hw, *, flipped: bool,
               out_dtype: Optional[torch.dtype] = None, residual: Optional[Tensor] = None) -> Tensor:
    """dX of a convolution.  dy: NHWC [n, oh, ow, cout]; wt: [cin, k*k*cout] from
    dgrad_weight (flipped for the stride-1 form).  in_hw = forward input (h, w)."""
    _contig(dy, "dy")
    n, oh, ow, cout = dy.shape
    h, w = in_hw
    cin = wt.shape[0]
    out = torch.empty((n, h, w, cin), device=dy.device, dtype=out_dtype or dy.dtype)
    d = L.GemmDesc()
    d.dtype = dtype_code(dy.dtype)
    d.M, d.N, d.K = n * h * w, cin, k * k * cout
    if wt.shape[1] != d.K:
        raise ValueError("conv_dgrad weight K mismatch")
    d.A, d.lda = dy.data_ptr(), cout
    d.B, d.ldb = wt.data_ptr(), wt.stride(0)
    d.C, d.ldc, d.c_dtype = out.data_ptr(), cin, dtype_code(out.dtype)
    d.alpha = 1.0
    if residual is not None:
        _contig(residual, "residual")
        d.residual, d.ldr, d.r_dtype = residual.data_ptr(), cin, dtype_code(residual.dtype)
    d.conv_n = n
    d.conv_k = k
    if flipped:
        if stride != 1:
            raise ValueError("flipped dgrad form is stride-1 only")
        d.conv_h, d.conv_w, d.conv_c = oh, ow, cout
        d.conv_stride, d.conv_pad, d.conv_oh, d.conv_ow = 1, k - 1 - pad, h, w
    else:
        d.conv_h, d.conv_w, d.conv_c = oh, ow, cout
        d.conv_stride, d.conv_pad, d.conv_oh, d.conv_ow = stride, pad, h, w
        d.conv_transposed = 1
    d.variant = options().gemm_variant
    check(L.lib().hv_gemm(C.byref(d), stream_ptr()), f"hv_gemm(conv dgrad {cout}->{cin} k{k} s{stride})")
    return out


def wgrad(a: Tensor, b: Tensor, *, out: Optional[Tensor] = None, accumulate: bool = False) -> Tensor:
    """C[N1, N2] (+)= a[P, N1]^T b[P, N2]  (fp32 result)."""
    _cuda(a, b)
    P, N1 = a.shape
    N2 = b.shape[1]
    if b.shape[0] != P or a.dtype != b.dtype:
        raise ValueError("wgrad operand mismatch")
    if out is None:
        out = torch.empty((N1, N2), device=a.device, dtype=torch.float32)
    lib = L.lib()
    work = _work(lib.hv_wgrad_work_floats(dtype_code(a.dtype), P, N1, N2), a.device)
    d = L.WgradDesc()
    d.dtype = dtype_code(a.dtype)
    d.P, d.N1, d.N2 = P, N1, N2
    d.A, d.lda = a.data_ptr(), a.stride(0)
    d.B, d.ldb = b.data_ptr(), b.stride(0)
    d.C, d.ldc = out.data_ptr(), out.stride(0)
    d.accumulate = int(accumulate)
    d.work = work.data_ptr()
    d.variant = options().wgrad_variant
    check(lib.hv_wgrad(C.byref(d), stream_ptr()), f"hv_wgrad P={P} N1={N1} N2={N2}")
    return out


def conv_wgrad(dy: Tensor, x: Tensor, k: int, stride: int, pad: int) -> Tensor:
    """dW [cout, k*k*cin] (columns (kh, kw, ci)) = dY^T im2col(X), fp32."""
    _contig(dy, "dy")
    _contig(x, "x")
    n, oh, ow, cout = dy.shape
    _, h, w, cin = x.shape
    N2 = k * k * cin
    P = n * oh * ow
    out = torch.empty((cout, N2), device=dy.device, dtype=torch.float32)
    lib = L.lib()
    work = _work(lib.hv_wgrad_work_floats(dtype_code(dy.dtype), P, cout, N2), dy.device)
    d = L.WgradDesc()
    d.dtype = dtype_code(dy.dtype)
    d.P, d.N1, d.N2 = P, cout, N2
    d.A, d.lda = dy.data_ptr(), cout
    d.B, d.ldb = x.data_ptr(), cin
    d.C, d.ldc = out.data_ptr(), N2
    d.work = work.data_ptr()
    d.conv_n, d.conv_h, d.conv_w, d.conv_c = n, h, w, cin
    d.conv_k, d.conv_stride, d.conv_pad, d.conv_oh, d.conv_ow = k, stride, pad, oh, ow
    d.variant = options().wgrad_variant
    check(lib.hv_wgrad(C.byref(d), stream_ptr()), f"hv_wgrad(conv {cin}->{cout} k{k})")
    return out


# ---------------------------------------------------------------------------- layouts
def dgrad_weight(w: Tensor, dtype: torch.dtype, flip: bool) -> Tensor:
    w = f32(w)
    cout, cin, k, _ = w.shape
    y = torch.empty((cin, k * k * cout), device=w.device, dtype=dtype)
    check(L.lib().hv_dgrad_weight_prep(w.data_ptr(), cout, cin, k, int(flip), dtype_code(dtype), y.data_ptr(),
                                       stream_ptr()), "hv_dgrad_weight_prep")
    return y


def transpose_cast(x: Tensor, dtype: torch.dtype) -> Tensor:
    x = f32(x)
    rows, cols = x.shape
    y = torch.empty((cols, rows), device=x.device, dtype=dtype)
    check(L.lib().hv_transpose_cast(x.data_ptr(), rows, cols, dtype_code(dtype), y.data_ptr(), stream_ptr()),
          "hv_transpose_cast")
    return y


def grad_out(p: Tensor) -> Optional[Tensor]:
    """Destination for parameter p's gradient: a fresh view of the trainer's flat gradient buffer
    the first time p's gradient is produced in a step (trainer.GradBuckets: autograd then stores that
    view as p.grad and no bucket copy runs), else None (no trainer, or a second contribution, which
    autograd accumulates into the first)."""
    claim = getattr(p, "_hv_grad_claim", None)
    return None if claim is None else claim()


def conv_grad_reorder(g: Tensor, cout: int, cin: int, k: int, out: Optional[Tensor] = None) -> Tensor:
    y = out if out is not None else torch.empty((cout, cin, k, k), device=g.device, dtype=torch.float32)
    check(L.lib().hv_conv_grad_reorder(_contig(g, "g").data_ptr(), cout, cin, k, y.data_ptr(), stream_ptr()),
          "hv_conv_grad_reorder")
    return y


def colsum(x: Tensor) -> Tensor:
    """fp32 column sums of a [rows, cols] (or NHWC, summed over all but the last dim) tensor."""
    _contig(x, "x")
    cols = x.shape[-1]
    rows = x.numel() // cols
    out = torch.empty(cols, device=x.device, dtype=torch.float32)
    work = _work(L.lib().hv_colsum_work_floats(rows, cols), x.device)
    check(L.lib().hv_colsum(dtype_code(x.dtype), x.data_ptr(), cols, rows, cols, out.data_ptr(), 0,
                            work.data_ptr(), stream_ptr()), "hv_colsum")
    return out


_colsum_pass = colsum      # gemm_train's fallback (its `colsum` argument shadows the function)


# ---------------------------------------------------------------------------- BatchNorm
def bn_stats(x: Tensor, eps: float, momentum: float, running_mean: Optional[Tensor],
             running_var: Optional[Tensor]):
    _contig(x, "x")
    c = x.shape[-1]
    rows = x.numel() // c
    mean = torch.empty(c, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    work = _work(L.lib().hv_bn_work_floats(rows, c), x.device)
    for t in (running_mean, running_var):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise TypeError("running stats must be contiguous fp32")
    check(L.lib().hv_bn_stats(dtype_code(x.dtype), x.data_ptr(), rows, c, eps, momentum, mean.data_ptr(),
                              rstd.data_ptr(), ptr(running_mean), ptr(running_var), work.data_ptr(), stream_ptr()),
          "hv_bn_stats")
    # running statistics were updated by the kernel: bump their versions like torch's in-place
    # update (VersionWatch: eval-mode frozen coefficients / captured graphs refold the BN)
    ran = [t for t in (running_mean, running_var) if t is not None]
    if ran:
        increment_version(ran)
    return mean, rstd


def bn_apply(x: Tensor, mean, rstd, gamma, beta, act: str) -> Tensor:
    c = x.shape[-1]
    y = torch.empty_like(x)
    g, b = f32(gamma), f32(beta)
    check(L.lib().hv_bn_apply(dtype_code(x.dtype), x.data_ptr(), x.numel() // c, c, mean.data_ptr(),
                              rstd.data_ptr(), ptr(g), ptr(b), L.ACT[act], y.data_ptr(), stream_ptr()), "hv_bn_apply")
    return y


def bn_backward(x: Tensor, dy: Tensor, mean, rstd, gamma, beta, act: str):
    _contig(dy, "dy")
    c = x.shape[-1]
    rows = x.numel() // c
    dx = torch.empty_like(x)
    dg = torch.empty(c, device=x.device, dtype=torch.float32)
    db = torch.empty_like(dg)
    g, b = f32(gamma), f32(beta)
    work = _work(L.lib().hv_bn_work_floats(rows, c), x.device)
    check(L.lib().hv_bn_backward(dtype_code(x.dtype), x.data_ptr(), dy.data_ptr(), rows, c, mean.data_ptr(),
                                 rstd.data_ptr(), ptr(g), ptr(b), L.ACT[act], dx.data_ptr(), dg.data_ptr(),
                                 db.data_ptr(), work.data_ptr(), stream_ptr()), "hv_bn_backward")
    return dx, dg, db


# ---------------------------------------------------------------------------- row norms
LN, RMS = 0, 1


def rownorm_train(mode: int, x: Tensor, eps: float, gamma=None, beta=None, drop_p: float = 0.0, seed: int = 0,
                  out_dtype: Optional[torch.dtype] = None, residual: Optional[Tensor] = None):
    _contig(x, "x")
    cols = x.shape[-1]
    rows = x.numel() // cols
    y = torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32) if mode == LN else None
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    g, b = f32(gamma), f32(beta)
    if residual is not None:
        _contig(residual, "residual")
        if residual.dtype != y.dtype:
            raise TypeError("rownorm_train: residual dtype must match the output")
    check(L.lib().hv_rownorm_train(mode, dtype_code(x.dtype), x.data_ptr(), rows, cols, eps, ptr(g), ptr(b),
                                   float(drop_p), int(seed) & 0xFFFFFFFF, seed_offset_ptr(), dtype_code(y.dtype),
                                   y.data_ptr(),
                                   ptr(residual), ptr(mean), rstd.data_ptr(), stream_ptr()), "hv_rownorm_train")
    return y, mean, rstd


def rownorm_backward(mode: int, x: Tensor, dy: Tensor, mean, rstd, gamma=None, drop_p: float = 0.0, seed: int = 0,
                     dx_dtype: Optional[torch.dtype] = None, dx_add: Optional[Tensor] = None,
                     param_grads: bool = True):
    _contig(x, "x")
    _contig(dy, "dy")
    cols = x.shape[-1]
    rows = x.numel() // cols
    dx = torch.empty(x.shape, device=x.device, dtype=dx_dtype or dy.dtype)
    if dx_add is not None:
        _contig(dx_add, "dx_add")
        if dx_add.dtype != dx.dtype:
            raise TypeError("rownorm_backward: dx_add dtype must match dx")
    dg = db = work = None
    if param_grads:
        dg = torch.empty(cols, device=x.device, dtype=torch.float32)
        db = torch.empty(cols, device=x.device, dtype=torch.float32) if mode == LN else None
        work = _work(L.lib().hv_rownorm_work_floats(rows, cols), x.device)
    g = f32(gamma)
    check(L.lib().hv_rownorm_backward(mode, dtype_code(x.dtype), x.data_ptr(), dtype_code(dy.dtype), dy.data_ptr(),
                                      rows, cols, ptr(mean), rstd.data_ptr(), ptr(g), float(drop_p),
                                      int(seed) & 0xFFFFFFFF, seed_offset_ptr(), dtype_code(dx.dtype), dx.data_ptr(),
                                      ptr(dx_add),
                                      ptr(dg), ptr(db), ptr(work), stream_ptr()), "hv_rownorm_backward")
    return dx, dg, db


def act_backward(dy: Tensor, pre: Tensor, act: str, drop_p: float = 0.0, seed: int = 0) -> Tensor:
    _contig(dy, "dy")
    _contig(pre, "pre")
    if dy.dtype != pre.dtype or dy.shape != pre.shape:
        raise ValueError("act_backward: dy/pre mismatch")
    out = torch.empty_like(dy)
    check(L.lib().hv_act_backward(dtype_code(dy.dtype), dy.data_ptr(), pre.data_ptr(), dy.numel(), L.ACT[act],
                                  float(drop_p), int(seed) & 0xFFFFFFFF, seed_offset_ptr(), out.data_ptr(),
                                  stream_ptr()),
          "hv_act_backward")
    return out


def dropout(x: Tensor, p: float, seed: int) -> Tensor:
    _contig(x, "x")
    y = torch.empty_like(x)
    check(L.lib().hv_dropout(dtype_code(x.dtype), x.data_ptr(), x.numel(), float(p), int(seed) & 0xFFFFFFFF,
                             seed_offset_ptr(), y.data_ptr(), stream_ptr()), "hv_dropout")
    return y


# ---------------------------------------------------------------------------- SE / pooling
def chan_dot(a: Tensor, b: Optional[Tensor]) -> Tensor:
    """[n, c] fp32 = sum over the middle (pixel) dims of a * b (b None: of a)."""
    _contig(a, "a")
    n, c = a.shape[0], a.shape[-1]
    hw = a.numel() // (n * c)
    if b is not None:
        _contig(b, "b")
        if b.shape != a.shape or b.dtype != a.dtype:
            raise ValueError("chan_dot operand mismatch")
    out = torch.empty((n, c), device=a.device, dtype=torch.float32)
    work = _work(L.lib().hv_chan_dot_work_floats(n, hw, c), a.device)
    check(L.lib().hv_chan_dot(dtype_code(a.dtype), a.data_ptr(), ptr(b), n, hw, c, out.data_ptr(), work.data_ptr(),
                              stream_ptr()), "hv_chan_dot")
    return out


def se_mlp_backward(pooled: Tensor, dgate: Tensor, w1, b1, w2, b2):
    n, c = pooled.shape
    cr = w1.shape[0]
    w1, b1, w2, b2 = map(f32, (w1, b1, w2, b2))
    dp = torch.empty_like(pooled)
    dw1 = torch.empty((cr, c), device=pooled.device, dtype=torch.float32)
    db1 = torch.empty(cr, device=pooled.device, dtype=torch.float32)
    dw2 = torch.empty((c, cr), device=pooled.device, dtype=torch.float32)
    db2 = torch.empty(c, device=pooled.device, dtype=torch.float32)
    work = _work(n * (c + 2 * cr), pooled.device)
    check(L.lib().hv_se_mlp_backward(pooled.data_ptr(), _contig(dgate, "dgate").data_ptr(), n, c, cr, w1.data_ptr(),
                                     b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), dp.data_ptr(), dw1.data_ptr(),
                                     db1.data_ptr(), dw2.data_ptr(), db2.data_ptr(), work.data_ptr(), stream_ptr()),
          "hv_se_mlp_backward")
    return dp, dw1, db1, dw2, db2


def se_backward_apply(dout: Tensor, gate: Tensor, dpooled: Tensor) -> Tensor:
    _contig(dout, "dout")
    n, c = dout.shape[0], dout.shape[-1]
    hw = dout.numel() // (n * c)
    dy = torch.empty_like(dout)
    check(L.lib().hv_se_backward_apply(dtype_code(dout.dtype), dout.data_ptr(), gate.data_ptr(), dpooled.data_ptr(),
                                       n, hw, c, dy.data_ptr(), stream_ptr()), "hv_se_backward_apply")
    return dy


def maxpool2x2_backward(x: Tensor, dy: Tensor) -> Tensor:
    n, h, w, c = x.shape
    dx = torch.empty_like(x)
    check(L.lib().hv_maxpool2x2_backward(dtype_code(x.dtype), _contig(x, "x").data_ptr(), _contig(dy, "dy").data_ptr(),
                                         n, h, w, c, dx.data_ptr(), stream_ptr()), "hv_maxpool2x2_backward")
    return dx


def upsample_backward(dy: Tensor, hb: int, wb: int) -> Tensor:
    n, h, w, c = dy.shape
    db = torch.empty((n, hb, wb, c), device=dy.device, dtype=dy.dtype)
    check(L.lib().hv_upsample_backward(dtype_code(dy.dtype), _contig(dy, "dy").data_ptr(), n, h, w, c, hb, wb,
                                       db.data_ptr(), stream_ptr()), "hv_upsample_backward")
    return db


def vit_assemble(x: Tensor, cls: Tensor, pos: Tensor) -> Tensor:
    n, t, d = x.shape
    cls, pos = f32(cls), f32(pos)
    z = torch.empty((n, t + 1, d), device=x.device, dtype=x.dtype)
    check(L.lib().hv_vit_assemble(dtype_code(x.dtype), _contig(x, "x").data_ptr(), cls.data_ptr(), pos.data_ptr(),
                                  n, t, d, z.data_ptr(), stream_ptr()), "hv_vit_assemble")
    return z


def vit_assemble_backward(dz: Tensor):
    n, t1, d = dz.shape
    dx = torch.empty((n, t1 - 1, d), device=dz.device, dtype=dz.dtype)
    dcls = torch.empty(d, device=dz.device, dtype=torch.float32)
    dpos = torch.empty((t1, d), device=dz.device, dtype=torch.float32)
    check(L.lib().hv_vit_assemble_backward(dtype_code(dz.dtype), _contig(dz, "dz").data_ptr(), n, t1 - 1, d,
                                           dx.data_ptr(), dcls.data_ptr(), dpos.data_ptr(), stream_ptr()),
          "hv_vit_assemble_backward")
    return dx, dcls, dpos


def scatter_rows(dy: Tensor, stride_rows: int) -> Tensor:
    n, c = dy.shape
    dx = torch.empty((n * stride_rows, c), device=dy.device, dtype=dy.dtype)
    check(L.lib().hv_scatter_rows(dtype_code(dy.dtype), _contig(dy, "dy").data_ptr(), stride_rows, n, c,
                                  dx.data_ptr(), stream_ptr()), "hv_scatter_rows")
    return dx


# ---------------------------------------------------------------------------- attention
# bf16 attention with head_dim 32 runs on the matrix cores (hv_attention_*_mfma); False = the
# scalar kernels (A/B and parity tests)
ATTN_MFMA = True


def _attn_mfma_ok(q: Tensor, heads: int) -> bool:
    return ATTN_MFMA and q.dtype == torch.bfloat16 and q.shape[-1] == 32 * heads


def attention_train(q: Tensor, k: Tensor, v: Tensor, heads: int, drop_p: float, seed: int):
    n, Lq, D = q.shape
    hd = D // heads
    o = torch.empty_like(q)
    lse = torch.empty((n, heads, Lq), device=q.device, dtype=torch.float32)
    if _attn_mfma_ok(q, heads):
        vt = torch.empty(L.lib().hv_attention_train_mfma_work_elems(n, Lq, heads), device=q.device, dtype=q.dtype)
        check(L.lib().hv_attention_train_mfma(_contig(q, "q").data_ptr(), _contig(k, "k").data_ptr(),
                                              _contig(v, "v").data_ptr(), o.data_ptr(), lse.data_ptr(), n, Lq, heads,
                                              hd ** -0.5, float(drop_p), int(seed) & 0xFFFFFFFF, seed_offset_ptr(),
                                              vt.data_ptr(),
                                              stream_ptr()), "hv_attention_train_mfma")
        return o, lse
    check(L.lib().hv_attention_train(dtype_code(q.dtype), _contig(q, "q").data_ptr(), _contig(k, "k").data_ptr(),
                                     _contig(v, "v").data_ptr(), o.data_ptr(), lse.data_ptr(), n, Lq, heads, hd,
                                     hd ** -0.5, float(drop_p), int(seed) & 0xFFFFFFFF, seed_offset_ptr(),
                                     stream_ptr()),
          "hv_attention_train")
    return o, lse


def attention_backward(q, k, v, o, do, lse, heads: int, drop_p: float, seed: int):
    n, Lq, D = q.shape
    hd = D // heads
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    if _attn_mfma_ok(q, heads) and do.dtype == q.dtype and o.dtype == q.dtype:
        te = L.lib().hv_attention_train_mfma_work_elems(n, Lq, heads)
        work = torch.empty(3 * te * 2 + n * heads * Lq * 4 + 64, device=q.device, dtype=torch.uint8)
        check(L.lib().hv_attention_backward_mfma(_contig(q, "q").data_ptr(), _contig(k, "k").data_ptr(),
                                                 _contig(v, "v").data_ptr(), _contig(o, "o").data_ptr(),
                                                 _contig(do, "dout").data_ptr(), lse.data_ptr(), n, Lq, heads,
                                                 hd ** -0.5, float(drop_p), int(seed) & 0xFFFFFFFF, seed_offset_ptr(),
                                                 dq.data_ptr(),
                                                 dk.data_ptr(), dv.data_ptr(), work.data_ptr(), stream_ptr()),
              "hv_attention_backward_mfma")
        return dq, dk, dv
    work = _work(n * heads * Lq, q.device)
    check(L.lib().hv_attention_backward(dtype_code(q.dtype), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                        _contig(do, "dout").data_ptr(), lse.data_ptr(), n, Lq, heads, hd, hd ** -0.5,
                                        float(drop_p), int(seed) & 0xFFFFFFFF, seed_offset_ptr(), dq.data_ptr(),
                                        dk.data_ptr(),
                                        dv.data_ptr(), work.data_ptr(), stream_ptr()), "hv_attention_backward")
    return dq, dk, dv


# ---------------------------------------------------------------------------- loss
def yolo_loss(logits: Tensor, targets: Tensor, A: int, lambdas, grad_dtype: Optional[torch.dtype] = None):
    """One scale of YOLOLoss.  logits NHWC [n, h, w, A*P]; targets [n, A, h, w, P] fp32.
    Returns (sums[6] fp32 device tensor, dlogits NHWC)."""
    _contig(logits, "logits")
    n, h, w, AP = logits.shape
    P = AP // A
    t = targets.detach().float().contiguous()
    if t.shape != (n, A, h, w, P):
        raise ValueError(f"yolo_loss: targets {tuple(t.shape)} != {(n, A, h, w, P)}")
    sums = torch.empty(6, device=logits.device, dtype=torch.float32)
    dl = torch.empty(logits.shape, device=logits.device, dtype=grad_dtype or logits.dtype)
    work = _work(L.lib().hv_yolo_loss_work_floats(n, h, w, A), logits.device)
    lc, lo, ln, lcl = lambdas
    check(L.lib().hv_yolo_loss(dtype_code(logits.dtype), logits.data_ptr(), t.data_ptr(), n, h, w, A, P, lc, lo, ln,
                               lcl, sums.data_ptr(), dtype_code(dl.dtype), dl.data_ptr(), work.data_ptr(),
                               stream_ptr()), "hv_yolo_loss")
    return sums, dl


def mhc_param_backward(dgc: Tensor, du: Tensor, h_pre_raw, gamma_pre, beta_pre, dwc_x: Tensor, dwc_h: Tensor,
                       h_post_raw):
    """One site's coefficient backward (hv_mhc_param_backward): returns dH_pre_raw, dgamma_pre,
    dbeta_pre, dH_res, dH_post_raw (fp32)."""
    D, Hd = dgc.shape
    dev = dgc.device
    hp, g, b, hq = f32(h_pre_raw), f32(gamma_pre), f32(beta_pre), f32(h_post_raw)
    dgc, du, dwc_x, dwc_h = (_contig(t, "grad") for t in (dgc, du.contiguous(), dwc_x, dwc_h))
    dhp = torch.empty((D, Hd), device=dev, dtype=torch.float32)
    dg = torch.empty(D, device=dev, dtype=torch.float32)
    db = torch.empty(D, device=dev, dtype=torch.float32)
    dhr = torch.empty((D, D), device=dev, dtype=torch.float32)
    dhq = torch.empty((Hd, D), device=dev, dtype=torch.float32)
    work = _work(L.lib().hv_mhc_param_backward_work_floats(D, Hd), dev)
    check(L.lib().hv_mhc_param_backward(D, Hd, dgc.data_ptr(), du.data_ptr(), hp.data_ptr(), g.data_ptr(),
                                        b.data_ptr(), dwc_x.data_ptr(), dwc_h.data_ptr(), hq.data_ptr(),
                                        dhp.data_ptr(), dg.data_ptr(), db.data_ptr(), dhr.data_ptr(), dhq.data_ptr(),
                                        work.data_ptr(), stream_ptr()), "hv_mhc_param_backward")
    return dhp, dg, db, dhr, dhq
