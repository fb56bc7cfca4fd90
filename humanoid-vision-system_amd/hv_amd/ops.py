"""Torch-tensor wrappers over the libhvs C ABI.

Every function launches HIP kernels on the current torch stream and returns freshly
allocated (caching-allocator) tensors; there is no CPU or eager-PyTorch fallback.
Activations are token-major: images are NHWC tensors [n, h, w, c] (contiguous), token
sequences are [rows, c].
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import _lib as L
from . import tables
from ._lib import check, dtype_code, ptr, stream_ptr
from .runtime import options

Tensor = torch.Tensor


def _cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("hv_amd ops require CUDA(HIP) tensors; there is no CPU path")


_KEEPALIVE: list = []     # stack of lists collecting the pinned sources of uploads under capture


class capture_keepalive:
    """While a HIP graph is being captured, a table upload becomes a memcpy NODE that re-reads its
    pinned host source on every replay: `with capture_keepalive(keep):` collects those sources
    (and the device tables) into `keep`, which the graph's owner holds as long as the graph."""

    def __init__(self, keep: list):
        self.keep = keep

    def __enter__(self):
        _KEEPALIVE.append(self.keep)
        return self.keep

    def __exit__(self, *exc):
        _KEEPALIVE.pop()
        return False


def keep_if_capturing(*objs) -> None:
    """Register host sources of an upload issued while the current stream captures a graph."""
    if _KEEPALIVE and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        _KEEPALIVE[-1].append(objs)


def upload_table(entries, device) -> Tensor:
    """ctypes struct array -> device bytes, asynchronously: a table upload never synchronises the
    host with the GPU, so it can sit inside a training forward/backward without draining the
    queue.  Outside a capture: pinned staging + non_blocking copy on the current stream.  Inside
    a graph capture (pinning new host memory is refused there): the bytes travel as kernel
    arguments (hv_write_bytes), recorded by value in the graph."""
    return upload_bytes(bytes(entries), device)


def upload_bytes(data: bytes, device, dtype: torch.dtype = torch.uint8) -> Tensor:
    """Host bytes -> a new device tensor of `dtype` (see upload_table)."""
    host = torch.frombuffer(bytearray(data), dtype=dtype) if data else torch.empty(0, dtype=dtype)
    if torch.device(device).type != "cuda":
        return host.to(device)
    if torch.cuda.is_current_stream_capturing():
        dev = torch.empty(host.shape, dtype=dtype, device=device)
        if host.numel():
            check(L.lib().hv_write_bytes(dev.data_ptr(), host.data_ptr(), host.numel() * host.element_size(),
                                         stream_ptr()), "hv_write_bytes")
        return dev
    host = host.pin_memory()
    return host.to(device, non_blocking=True)


def _contig(t: Tensor, name: str) -> Tensor:
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


# ---------------------------------------------------------------------------- GEMM
# Split-K is opt-in (HVOptions.splitk): measured no gain (profiles/r02/splitk_ab.txt) -- with a
# separate reduce launch the split GEMM + reduce (6.1 + 5.4 us) cost what the un-split kernel
# does (10.1 us) at B=1; with the reduction fused into the last-arriving workgroup the
# agent-scope release/acquire (L2 write-back + invalidate on every workgroup) made it 31 us.
_SPLITK_COUNTERS: dict = {}
SPLITK_MAX_TILES = 4096                                      # HV_SPLITK_MAX_TILES


def _splitk_counters(device) -> Tensor:
    """Per-(device, stream) tile arrival counters of the split-K kernel: zeroed once, and every
    launch leaves them zero (its last workgroup per tile resets its counter); launches on one
    stream are ordered, so they can share them."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    c = _SPLITK_COUNTERS.get(key)
    if c is None:
        c = torch.zeros(SPLITK_MAX_TILES, device=device, dtype=torch.int32)
        _SPLITK_COUNTERS[key] = c
    return c


def _splitk(d, M: int, N: int, K: int, dtype: torch.dtype, device) -> Optional[Tensor]:
    """Split-K for small output grids with long contractions (B=1 streaming: the ViT's 401-token
    GEMMs, the coarse FPN / head convs; the 16-row final-fusion GEMMs at any batch): the bf16
    LDS-DMA kernel has too few 64x64 output tiles to fill 256 CUs, so each tile's K-tiles are
    split over `splitk` workgroups (>= 4 K-tiles each); the last workgroup of a tile to finish
    sums the fp32 partials in slice order and runs the epilogue (deterministic).  Returns the workspace
    (kept alive by the caller until the launch is enqueued) or None."""
    o = options()
    if not (o.splitk or M <= o.splitk_small_m) or dtype != torch.bfloat16 or K % 64:
        return None
    tiles = -(-M // 64) * -(-N // 64)
    if tiles >= 192:
        return None
    splits = min(K // 256, max(2, 384 // tiles), 64)
    if splits < 2:
        return None
    work = torch.empty(splits * M * N, device=device, dtype=torch.float32)
    d.splitk_work, d.splitk_count, d.splitk = work.data_ptr(), _splitk_counters(device).data_ptr(), splits
    return work


def gemm(a: Tensor, b: Tensor, *, bias: Optional[Tensor] = None, scale: Optional[Tensor] = None,
         act: str = "none", alpha: float = 1.0, residual: Optional[Tensor] = None,
         a_mean: Optional[Tensor] = None, a_rstd: Optional[Tensor] = None,
         a2: Optional[Tensor] = None, out_dtype: Optional[torch.dtype] = None,
         out: Optional[Tensor] = None, residual_mod: int = 0, b_colsum: Optional[Tensor] = None,
         variant: Optional[int] = None) -> Tensor:
    """C = act((a' @ b^T) * alpha * scale + bias) + residual.

    a: [M, K1] (row stride may exceed K1), b: [N, K] with K = K1 (+ K2 if a2 [M, K2] given).
    a_mean/a_rstd: per-row LayerNorm statistics of a (applied on load, or -- given
    b_colsum = b.sum(1) in fp32 -- after the product as rstd * (acc - mean * b_colsum)).
    variant: kernel selection for this launch (HV_GV_* bits, _lib.GV_*); None = the forward's
    HVOptions.gemm_variant (0 = automatic).
    """
    _cuda(a, b)
    if a.dim() != 2 or b.dim() != 2 or a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("gemm expects 2-D row-major operands")
    if a.dtype != b.dtype or (a2 is not None and a2.dtype != a.dtype):
        raise TypeError("gemm operands must share a dtype")
    M, K1 = a.shape
    K = K1 + (a2.shape[1] if a2 is not None else 0)
    N = b.shape[0]
    if b.shape[1] != K:
        raise ValueError(f"gemm K mismatch: a {tuple(a.shape)} a2 {None if a2 is None else tuple(a2.shape)} b {tuple(b.shape)}")
    od = out_dtype or a.dtype
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=od)
    d = L.GemmDesc()
    d.dtype = dtype_code(a.dtype)
    d.M, d.N, d.K = M, N, K
    d.A, d.lda = a.data_ptr(), a.stride(0)
    if a2 is not None:
        if a2.shape[0] != M or a2.stride(1) != 1:
            raise ValueError("a2 must be [M, K2] row-major")
        d.A2, d.lda2, d.k1 = a2.data_ptr(), a2.stride(0), K1
    d.B, d.ldb = b.data_ptr(), b.stride(0)
    d.C, d.ldc, d.c_dtype = out.data_ptr(), out.stride(0), dtype_code(out.dtype)
    d.a_mean, d.a_rstd = ptr(a_mean), ptr(a_rstd)
    d.b_colsum = ptr(b_colsum) if a_mean is not None else None
    d.scale, d.bias = ptr(scale), ptr(bias)
    d.act = L.ACT[act]
    d.alpha = alpha
    if residual is not None:
        d.residual, d.ldr, d.r_dtype = residual.data_ptr(), residual.stride(0), dtype_code(residual.dtype)
        d.r_mod = residual_mod
    d.variant = options().gemm_variant if variant is None else variant
    work = _splitk(d, M, N, K, a.dtype, a.device)      # noqa: F841  (alive until enqueued)
    check(L.lib().hv_gemm(C.byref(d), stream_ptr()), f"hv_gemm M={M} N={N} K={K}")
    return out


def conv2d(x: Tensor, w: Tensor, k: int, stride: int, pad: int, *, scale=None, bias=None,
           act: str = "none", residual: Optional[Tensor] = None,
           out_dtype: Optional[torch.dtype] = None, variant: Optional[int] = None) -> Tensor:
    """Implicit-GEMM convolution. x: NHWC [n, h, w, c]; w: [cout, k*k*c] (from conv_weight_prep)."""
    _cuda(x, w)
    _contig(x, "conv input")
    n, h, wd, c = x.shape
    oh = (h + 2 * pad - k) // stride + 1
    ow = (wd + 2 * pad - k) // stride + 1
    cout = w.shape[0]
    out = torch.empty((n, oh, ow, cout), device=x.device, dtype=out_dtype or x.dtype)
    d = L.GemmDesc()
    d.dtype = dtype_code(x.dtype)
    d.M, d.N, d.K = n * oh * ow, cout, k * k * c
    if w.shape[1] != d.K:
        raise ValueError(f"conv weight K {w.shape[1]} != {d.K}")
    d.A, d.lda = x.data_ptr(), c
    d.B, d.ldb = w.data_ptr(), w.stride(0)
    d.C, d.ldc, d.c_dtype = out.data_ptr(), cout, dtype_code(out.dtype)
    d.scale, d.bias = ptr(scale), ptr(bias)
    d.act = L.ACT[act]
    d.alpha = 1.0
    if residual is not None:
        _contig(residual, "residual")
        d.residual, d.ldr, d.r_dtype = residual.data_ptr(), cout, dtype_code(residual.dtype)
    d.conv_n, d.conv_h, d.conv_w, d.conv_c = n, h, wd, c
    d.conv_k, d.conv_stride, d.conv_pad, d.conv_oh, d.conv_ow = k, stride, pad, oh, ow
    d.variant = options().gemm_variant if variant is None else variant
    work = _splitk(d, d.M, cout, d.K, x.dtype, x.device)   # noqa: F841  (alive until enqueued)
    check(L.lib().hv_gemm(C.byref(d), stream_ptr()), f"hv_gemm(conv {c}->{cout} k{k} s{stride})")
    return out


def conv_stem(img: Tensor, w: Tensor, k: int, stride: int, pad: int, dtype: torch.dtype, *, scale=None,
              bias=None, act: str = "none", nhwc: bool = False) -> Optional[Tensor]:
    """Direct 3x3 conv of a 3-channel image -> NHWC `dtype` (hv_conv_stem): img is the NCHW fp32
    batch (nhwc=False) or an NHWC `dtype` tensor (nhwc=True).  None when the shape is not one
    the direct kernel covers (the caller uses conv2d)."""
    _cuda(img, w)
    if img.dim() != 4 or not img.is_contiguous() or w.dtype != dtype:
        return None
    if nhwc:
        n, h, wd, c = img.shape
        if img.dtype != dtype:
            return None
    else:
        n, c, h, wd = img.shape
        if img.dtype != torch.float32:
            return None
    oh = (h + 2 * pad - k) // stride + 1
    ow = (wd + 2 * pad - k) // stride + 1
    cout = w.shape[0]
    if c != 3 or k != 3 or cout not in (32, 64) or w.shape[1] < 27 or w.stride(1) != 1 or oh <= 0 or ow <= 0:
        return None
    out = torch.empty((n, oh, ow, cout), device=img.device, dtype=dtype)
    rc = L.lib().hv_conv_stem(dtype_code(dtype), img.data_ptr(), int(nhwc), n, c, h, wd, k, stride, pad,
                              w.data_ptr(), w.stride(0), cout, ptr(scale), ptr(bias), L.ACT[act], out.data_ptr(),
                              stream_ptr())
    if rc == -2:          # HV_EUNSUPPORTED
        return None
    check(rc, "hv_conv_stem")
    return out


# ---------------------------------------------------------------------------- parameters
def conv_weight_prep(w: Tensor, dtype: torch.dtype, scale: Optional[Tensor] = None) -> Tensor:
    """[cout, cin, k, k] fp32 -> [cout, k*k*cin] (K padded to a 16-byte multiple)."""
    _cuda(w)
    w = w.detach().float().contiguous()
    cout, cin, k, _ = w.shape
    kk = k * k * cin
    epc = 8 if dtype == torch.bfloat16 else 4
    kp = (kk + epc - 1) // epc * epc
    if kp == kk:
        out = torch.empty((cout, kk), device=w.device, dtype=dtype)
        check(L.lib().hv_conv_weight_prep(w.data_ptr(), cout, cin, k, ptr(scale), dtype_code(dtype),
                                          out.data_ptr(), stream_ptr()), "hv_conv_weight_prep")
        return out
    tmp = torch.empty((cout, kk), device=w.device, dtype=dtype)
    check(L.lib().hv_conv_weight_prep(w.data_ptr(), cout, cin, k, ptr(scale), dtype_code(dtype),
                                      tmp.data_ptr(), stream_ptr()), "hv_conv_weight_prep")
    out = torch.zeros((cout, kp), device=w.device, dtype=dtype)
    out[:, :kk].copy_(tmp)
    return out[:, :kk]


def bn_fold(c: int, device, gamma=None, beta=None, mean=None, var=None, conv_bias=None,
            eps: float = 1e-5):
    s = torch.empty(c, device=device, dtype=torch.float32)
    b = torch.empty(c, device=device, dtype=torch.float32)
    f = lambda t: None if t is None else t.detach().float().contiguous()  # noqa: E731
    gamma, beta, mean, var, conv_bias = map(f, (gamma, beta, mean, var, conv_bias))
    check(L.lib().hv_bn_fold(c, ptr(gamma), ptr(beta), ptr(mean), ptr(var), ptr(conv_bias), eps,
                             s.data_ptr(), b.data_ptr(), stream_ptr()), "hv_bn_fold")
    return s, b


def cast(x: Tensor, dtype: torch.dtype) -> Tensor:
    _cuda(x)
    x = x.detach()
    if x.dtype != torch.float32:
        raise TypeError("cast expects fp32 input")
    x = x.contiguous()
    if dtype == torch.float32:
        return x
    y = torch.empty(x.shape, device=x.device, dtype=dtype)
    check(L.lib().hv_cast(x.data_ptr(), x.numel(), dtype_code(dtype), y.data_ptr(), stream_ptr()), "hv_cast")
    return y


def f32(t: Optional[Tensor]) -> Optional[Tensor]:
    return None if t is None else t.detach().float().contiguous()


def _mhc_variant(D: int, T: Optional[int], variant: Optional[int], Hd: Optional[int] = None, nsites: int = 1) -> int:
    """D = 256 sites take the split-hidden fused kernel (HV_MV_SPLIT256) automatically only from
    HVOptions.mhc256_min_tokens tokens: one 64-token group per workgroup, so small grids leave CUs
    idle and the unfused chain (the ViT's grouped q / k / v GEMM1) wins -- per launch 0.421 vs
    0.482 ms at T = 102,400, 0.124 vs 0.138 at 25,600, equal at 6,416 / 401; in-model with EVERY
    D = 256 site fused: B=16 19.90 vs 19.18 ms, B=1 9.0 vs 7.05 ms (profiles/r04/mhc256_ab.txt)."""
    o = options()
    v = o.mhc_variant if variant is None else variant
    if v == 0 and T is not None and o.mhc_tok:
        v = _tok_variant(D, Hd, T, nsites)
    if v == 0 and D == 256 and T is not None and T >= o.mhc256_min_tokens:
        v = L.MV_SPLIT256
    return v


# Token-tile kernel (hv_mhc_tok.hip) policy, from the per-launch A/B (tools/mhc_tok_ab.py,
# profiles/r05/mhc_tok_ab.txt): (D, Hd) -> largest token count it takes.  (256, 512): 23 us at
# T = 401 / 33 at 6,416 / 116 at 25,600 vs the chain's 59 / 62 / 136 and the split-hidden kernel's
# 124 at 25,600; (128, 512): 26 vs 58-60 us at 6,400, but the split-hidden kernel wins from 25,600
# (64 vs 94 us); (256, 1024) ties the chain at 1,600 and loses at 6,400: not taken.  Every
# workgroup streams all of a site's weights, so 16-token tiles (twice the workgroups) win while
# the grid fits the 256 CUs in one round, 32-token tiles (half the weight traffic per token) after.
TOK_MAX_T = {(128, 512): 12800, (256, 512): 51200, (256, 1024): 2048}   # (256, 1024): hidden split only
TOK_CUS = 256
TOK_SPLIT4_CUS = 256      # (256, 1024): the 4-way split while 4 x tiles <= this (else 2-way)


def _tok_variant(D: int, Hd: Optional[int], T: int, nsites: int = 1) -> int:
    if Hd is None or T > TOK_MAX_T.get((D, Hd), -1):
        return 0
    v = L.MV_TOK
    tiles16 = -(-T // 16) * nsites
    if tiles16 <= TOK_CUS:
        v |= L.MV_TOK16
        # at most a quarter as many tiles as CUs: each tile's hidden units split over 4
        # workgroups (per launch, profiles/r05/mhc_toksplit_ab.txt: T = 401 21.1 vs 23.2 us, T = 16
        # 17.6 vs 22.7; in-model B=1 frozen p50 4.20-4.25 vs 4.43-4.46 ms).  The 2-way split is
        # kept for tests only: 24.5 vs 25.1 us on the grouped q / k / v at T = 401, and slower
        # than the unsplit kernel at T = 1,604 (26.9 vs 24.0)
        if (D, Hd) == (256, 512) and options().mhc_tok_split and 4 * tiles16 <= TOK_CUS:
            v |= L.MV_TOKSPLIT4
    if (D, Hd) == (256, 1024):
        # (256, 1024) only split (5.9 MB of weights per unsplit workgroup ties the chain): T = 400
        # 32.6 (4-way) vs 57.7 us chain, T = 1,600 48.7 (2-way) vs 62.6 us
        if not (options().mhc_tok_split and v & L.MV_TOK16 and 2 * tiles16 <= TOK_CUS):
            return 0
        v |= L.MV_TOKSPLIT4 if 4 * tiles16 <= TOK_SPLIT4_CUS else L.MV_TOKSPLIT2
    return v




_TOKSPLIT_COUNTERS: dict = {}
TOKSPLIT_MAX_TILES = 4096


def _tok_split_buffers(a, n: int, T: int, D: int, variant: int, device):
    """Workspace + arrival counters of a hidden-split token-tile launch (hv_kernels.h
    HV_MV_TOKSPLIT*), set on the first site's args.  Counters are per (device, stream), zero and
    left zero by every launch; launches on one stream are ordered, so they can share them.
    Returns the workspace (kept alive by the caller until the launch is enqueued)."""
    nspl = 4 if variant & L.MV_TOKSPLIT4 else (2 if variant & L.MV_TOKSPLIT2 else 1)
    if nspl == 1:
        return None
    tiles = -(-T // 16) * n
    if tiles > TOKSPLIT_MAX_TILES:
        raise ValueError(f"token-tile split: {tiles} tiles > {TOKSPLIT_MAX_TILES}")
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    c = _TOKSPLIT_COUNTERS.get(key)
    if c is None:
        c = _TOKSPLIT_COUNTERS[key] = torch.zeros(TOKSPLIT_MAX_TILES, device=device, dtype=torch.int32)
    work = torch.empty(tiles * nspl * 16 * D, device=device, dtype=torch.float32)
    a.split_work, a.split_count = work.data_ptr(), c.data_ptr()
    return work


def mhc_fused_supported(D: int, Hd: int, dtype: torch.dtype, variant: Optional[int] = None,
                        T: Optional[int] = None) -> bool:
    """T: the site's token count (None = the token-count-independent answer)."""
    v = _mhc_variant(D, T, variant, Hd)
    return dtype in (torch.float32, torch.bfloat16) and bool(L.lib().hv_mhc_fused_supported(D, Hd, dtype_code(dtype), v))


def mhc_fused(x: Tensor, a1t, c1, w2, b2, wct, g_post, b_post, residual: Optional[Tensor] = None,
              variant: Optional[int] = None) -> Tensor:
    """One-launch mHC token chain (bf16) for x [T, D]; see hv_mhc_fused in hv_kernels.h.
    variant: HV_MV_* bits for this launch (None = the forward's HVOptions.mhc_variant)."""
    _contig(x, "x")
    T, D = x.shape
    Hd = w2.shape[0]
    if a1t.shape != (2 * Hd, D) or w2.shape != (Hd, 2 * Hd) or wct.shape != (D, D + Hd):
        raise ValueError("mhc_fused: coefficient shapes do not match x")
    for t in (a1t, w2, wct):
        _contig(t, "coefficient")
    if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype or not residual.is_contiguous()):
        raise ValueError("mhc_fused: residual must match x")
    out = torch.empty_like(x)
    v = _mhc_variant(D, T, variant, Hd)
    a = L.MhcFusedArgs(dtype_code(x.dtype), D, Hd, T, x.data_ptr(), a1t.data_ptr(), c1.data_ptr(), w2.data_ptr(),
                       b2.data_ptr(), wct.data_ptr(), g_post.data_ptr(), b_post.data_ptr(), ptr(residual),
                       out.data_ptr(), v, 0)
    work = _tok_split_buffers(a, 1, T, D, v, x.device)     # noqa: F841  (alive until enqueued)
    check(L.lib().hv_mhc_fused(C.byref(a), stream_ptr()), f"hv_mhc_fused D={D}")
    return out


def mhc_group_variant(D: int, Hd: int, T: int, n: int, dtype: torch.dtype, variant: Optional[int] = None) -> int:
    """HV_MV_* of a grouped launch of n sites (0: no grouped fused kernel for this shape)."""
    if dtype != torch.bfloat16:
        return 0
    v = _mhc_variant(D, T, variant, Hd, n)
    if not v & L.MV_TOK or not L.lib().hv_mhc_fused_supported(D, Hd, dtype_code(dtype), v):
        return 0
    return v


def mhc_fused_group(x: Tensor, plans, variant: int) -> list:
    """n <= 3 mHC chains on the SAME x [T, D] (q / k / v) in one launch (hv_mhc_fused_group);
    plans: manifold.MhcPlan (folded), variant from mhc_group_variant."""
    _contig(x, "x")
    T, D = x.shape
    n = len(plans)
    arr = (L.MhcFusedArgs * n)()
    outs = []
    for i, p in enumerate(plans):
        Hd = p.w2.shape[0]
        if p.b1.shape != (2 * Hd, D) or p.w2.shape != (Hd, 2 * Hd) or p.wct.shape != (D, D + Hd) or not p.fold:
            raise ValueError("mhc_fused_group: coefficient shapes do not match x")
        o = torch.empty_like(x)
        outs.append(o)
        arr[i] = L.MhcFusedArgs(dtype_code(x.dtype), D, Hd, T, x.data_ptr(), p.b1.data_ptr(), p.c1.data_ptr(),
                                p.w2.data_ptr(), p.bias2.data_ptr(), p.wct.data_ptr(), p.g_post.data_ptr(),
                                p.b_post.data_ptr(), None, o.data_ptr(), variant, 0)
    work = _tok_split_buffers(arr[0], n, T, D, variant, x.device)     # noqa: F841  (alive until enqueued)
    check(L.lib().hv_mhc_fused_group(arr, n, stream_ptr()), f"hv_mhc_fused_group D={D} n={n}")
    return outs


def gemv(w: Tensor, x: Tensor, b: Optional[Tensor] = None) -> Tensor:
    """fp32 y = w @ x + b for w [N, K], x [K]."""
    w, x, b = f32(w), f32(x), f32(b)
    N, K = w.shape
    if x.numel() != K or (b is not None and b.numel() != N):
        raise ValueError("gemv shape mismatch")
    y = torch.empty(N, device=w.device, dtype=torch.float32)
    check(L.lib().hv_gemv(w.data_ptr(), x.data_ptr(), ptr(b), N, K, y.data_ptr(), stream_ptr()), "hv_gemv")
    return y


# ---------------------------------------------------------------------------- norms
def row_stats(x: Tensor, eps: float = 1e-5):
    _cuda(x)
    rows, cols = x.shape
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    check(L.lib().hv_row_stats(dtype_code(x.dtype), x.data_ptr(), x.stride(0), rows, cols, eps,
                               mean.data_ptr(), rstd.data_ptr(), stream_ptr()), "hv_row_stats")
    return mean, rstd


def layernorm(x: Tensor, gamma: Optional[Tensor], beta: Optional[Tensor], eps: float = 1e-5,
              out_dtype: Optional[torch.dtype] = None, residual: Optional[Tensor] = None) -> Tensor:
    _cuda(x)
    _contig(x, "layernorm input")
    rows, cols = x.reshape(-1, x.shape[-1]).shape
    y = torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    if residual is not None:
        _contig(residual, "residual")
    check(L.lib().hv_layernorm(dtype_code(x.dtype), x.data_ptr(), rows, cols, eps, ptr(gamma), ptr(beta),
                               dtype_code(y.dtype), y.data_ptr(), ptr(residual),
                               dtype_code(residual.dtype) if residual is not None else 0, stream_ptr()),
          "hv_layernorm")
    return y


def rmsnorm(x: Tensor, scale: Tensor, eps: float = 1e-8) -> Tensor:
    _cuda(x)
    _contig(x, "rmsnorm input")
    cols = x.shape[-1]
    y = torch.empty_like(x)
    check(L.lib().hv_rmsnorm(dtype_code(x.dtype), x.data_ptr(), x.numel() // cols, cols, eps,
                             scale.data_ptr(), y.data_ptr(), stream_ptr()), "hv_rmsnorm")
    return y


# ---------------------------------------------------------------------------- sinkhorn
class SinkhornGroup:
    """A device table of Sinkhorn problems launched together (hv_sinkhorn_group_forward).

    Buffers (outputs, workspaces, the table itself) are allocated once per group and reused
    on every run, so the table's pointers stay valid.
    """

    def __init__(self, raws, iters, device, eps: float = 1e-8, tau: float = 1.0, hists=None):
        self.raws = list(raws)
        self.iters = list(iters)
        lib = L.lib()
        n_e = len(self.raws)
        self.outs, self.hists, self.works = [], [], []
        entries = (L.SinkhornEntry * n_e)()
        rs = rbs = cs = 0
        for i, (raw, it) in enumerate(zip(self.raws, self.iters)):
            if raw.dim() == 2:
                b, n, m = 1, raw.shape[0], raw.shape[1]
            else:
                b, n, m = raw.shape
            if m > 2048:
                raise ValueError("hv sinkhorn supports up to 2048 columns")
            out = torch.empty((b, n, m), device=device, dtype=torch.float32)
            hist = hists[i] if hists is not None else torch.zeros(max(it, 1), device=device, dtype=torch.float32)
            work = torch.empty(lib.hv_sinkhorn_work_floats(b, n, m, it), device=device, dtype=torch.float32)
            self.outs.append(out)
            self.hists.append(hist)
            self.works.append(work)
            e = entries[i]
            e.raw = 0  # filled per run (raw may be re-materialised)
            e.out, e.history, e.work = out.data_ptr(), hist.data_ptr(), work.data_ptr()
            e.batch, e.n, e.m, e.iters, e.eps, e.tau = b, n, m, it, eps, tau
            e.row_start, e.row_block_start, e.col_start = rs, rbs, cs
            rs += b * n
            rbs += b * ((n + 15) // 16)
            cs += b * m
        self.entries = entries
        self.totals = (rs, rbs, cs)
        small = [e.batch == 1 and e.n <= 256 and e.m <= 256 for e in entries]
        self.has_small, self.has_large = any(small), not all(small)
        # the grouped passes get a table of the large entries alone (own prefix sums): no idle
        # blocks for the small ones and a short entry search; same work pointers as the full table
        self._large_idx = [i for i, sm in enumerate(small) if not sm]
        self.entries_large = (L.SinkhornEntry * max(1, len(self._large_idx)))()
        rs_l = rbs_l = cs_l = 0
        for k, i in enumerate(self._large_idx):
            el = self.entries_large[k]
            C.memmove(C.addressof(el), C.addressof(entries[i]), C.sizeof(el))
            el.row_start, el.row_block_start, el.col_start = rs_l, rbs_l, cs_l
            rs_l += el.batch * el.n
            rbs_l += el.batch * ((el.n + 15) // 16)
            cs_l += el.batch * el.m
        self.totals_large = (rs_l, rbs_l, cs_l)
        self.table = None
        self.table_large = None
        self._raw_ptrs = None
        self.device = device

    def run(self, raws=None):
        raws = self.raws if raws is None else raws
        rp = tuple(r.data_ptr() for r in raws)
        if rp != self._raw_ptrs:
            for e, p in zip(self.entries, rp):
                e.raw = p
            for k, i in enumerate(self._large_idx):
                self.entries_large[k].raw = rp[i]
            self.table = tables.upload(self.entries, self.device, self, "entries")
            if self.has_large:
                self.table_large = tables.upload(self.entries_large, self.device, self, "entries_large")
            self._raw_ptrs = rp
        lib = L.lib()
        mx = max(self.iters)

        if self.has_small and mx > lib.hv_sinkhorn_small_max_iters():
            # too many iterations for the single-workgroup kernel's LDS history: every entry
            # through the grouped passes (part 0 on the full table)
            rs, rbs, cs = self.totals
            check(lib.hv_sinkhorn_group_forward_part(self.table.data_ptr(), len(self.entries), rs, rbs, cs, mx, 0,
                                                     stream_ptr()), "hv_sinkhorn_group_forward")
            return self.outs
        if self.has_small:          # small matrices: one workgroup each, all iterations in one launch
            rs, rbs, cs = self.totals
            check(lib.hv_sinkhorn_group_forward_part(self.table.data_ptr(), len(self.entries), rs, rbs, cs, mx, 1,
                                                     stream_ptr()), "hv_sinkhorn_group_forward_part")
        if self.has_large:          # the grouped row / column passes over the large entries' table
            rs, rbs, cs = self.totals_large
            check(lib.hv_sinkhorn_group_forward_part(self.table_large.data_ptr(), len(self._large_idx), rs, rbs,
                                                     cs, mx, 2, stream_ptr()), "hv_sinkhorn_group_forward_part")
        return self.outs


    def backward(self, douts):
        """Grouped reverse sweep (hv_sinkhorn_group_backward): dL/draw for dL/dM = douts
        (None entries count as zero).  Must follow run() with the same raws."""
        lib = L.lib()
        n_e = len(self.entries)
        bent = (L.SinkhornBwdEntry * n_e)()
        draws, keep = [], []
        for i, (e, raw) in enumerate(zip(self.entries, self.raws)):
            b, n, m = e.batch, e.n, e.m
            d = douts[i]
            d = torch.zeros((b, n, m), device=self.device, dtype=torch.float32) if d is None \
                else d.detach().float().contiguous()
            dr = torch.empty((b, n, m), device=self.device, dtype=torch.float32)
            bw = torch.empty(lib.hv_sinkhorn_bwd_work_floats(b, n, m), device=self.device, dtype=torch.float32)
            be = bent[i]
            be.fwd = e
            be.dout, be.draw, be.bwork = d.data_ptr(), dr.data_ptr(), bw.data_ptr()
            keep += [d, bw]
            draws.append(dr.view(raw.shape))
        table = upload_table(bent, self.device)
        rs, rbs, cs = self.totals
        check(lib.hv_sinkhorn_group_backward(table.data_ptr(), n_e, rs, rbs, cs, max(self.iters), stream_ptr()),
              "hv_sinkhorn_group_backward")
        return draws


def sinkhorn(raw: Tensor, iters: int, eps: float = 1e-8, tau: float = 1.0):
    """One Sinkhorn-Knopp projection ([n, m] or [b, n, m]); returns (M, history)."""
    _cuda(raw)
    r = raw.detach().float().contiguous()
    g = SinkhornGroup([r], [iters], raw.device, eps, tau)
    out = g.run([r])[0]
    return (out.squeeze(0) if raw.dim() == 2 else out), g.hists[0][:iters]


# ---------------------------------------------------------------------------- mHC prep
def mhc_prep(h_pre_raw, h_post_raw, h_res, gamma_pre, beta_pre, gc_transposed: bool):
    D, Hd = h_pre_raw.shape
    dev = h_pre_raw.device
    gc = torch.empty((Hd, D) if gc_transposed else (D, Hd), device=dev, dtype=torch.float32)
    u = torch.empty(Hd, device=dev, dtype=torch.float32)
    wct = torch.empty((D, D + Hd), device=dev, dtype=torch.float32)
    rm = torch.empty(D + Hd, device=dev, dtype=torch.float32)
    args = [f32(h_pre_raw), f32(h_post_raw), h_res.contiguous(), f32(gamma_pre), f32(beta_pre)]
    check(L.lib().hv_mhc_prep(D, Hd, *[a.data_ptr() for a in args], gc.data_ptr(), int(gc_transposed),
                              u.data_ptr(), wct.data_ptr(), rm.data_ptr(), stream_ptr()), "hv_mhc_prep")
    return gc, u, wct


# ---------------------------------------------------------------------------- pointwise
def nchw_to_nhwc(x: Tensor, dtype: torch.dtype) -> Tensor:
    _cuda(x)
    x = x.float().contiguous()
    n, c, h, w = x.shape
    y = torch.empty((n, h, w, c), device=x.device, dtype=dtype)
    check(L.lib().hv_nchw_to_nhwc(x.data_ptr(), n, c, h, w, dtype_code(dtype), y.data_ptr(), stream_ptr()),
          "hv_nchw_to_nhwc")
    return y


def maxpool2x2(x: Tensor, gate: Optional[Tensor] = None) -> Tensor:
    """MaxPool2d(2, 2) on NHWC; with gate [n, c] fp32 (SE sigmoid gate, > 0) it returns
    maxpool(x * gate) in one pass (bitwise equal to scale_residual followed by the pool)."""
    n, h, w, c = x.shape
    y = torch.empty((n, h // 2, w // 2, c), device=x.device, dtype=x.dtype)
    _contig(x, "x")
    if gate is not None:
        _contig(gate, "gate")
        if gate.dtype != torch.float32 or gate.numel() != n * c:
            raise ValueError("maxpool2x2 gate must be fp32 [n, c]")
    if c % 8 == 0 and (x.data_ptr() | y.data_ptr() | (gate.data_ptr() if gate is not None else 0)) % 16 == 0:
        check(L.lib().hv_scale_maxpool2x2(dtype_code(x.dtype), x.data_ptr(), ptr(gate), n, h, w, c, y.data_ptr(),
                                          stream_ptr()), "hv_scale_maxpool2x2")
        return y
    if gate is not None:
        x = scale_residual(x, gate, None)
    check(L.lib().hv_maxpool2x2(dtype_code(x.dtype), _contig(x, "x").data_ptr(), n, h, w, c, y.data_ptr(),
                                stream_ptr()), "hv_maxpool2x2")
    return y


def channel_mean(x: Tensor) -> Tensor:
    """NHWC [n, h, w, c] (or [n, p, c]) -> fp32 [n, c]."""
    _contig(x, "x")
    n, c = x.shape[0], x.shape[-1]
    hw = x.numel() // (n * c)
    out = torch.empty((n, c), device=x.device, dtype=torch.float32)
    work = torch.empty(L.lib().hv_channel_mean_work_floats(n, hw, c), device=x.device, dtype=torch.float32)
    check(L.lib().hv_channel_mean(dtype_code(x.dtype), x.data_ptr(), n, hw, c, out.data_ptr(), work.data_ptr(),
                                  stream_ptr()), "hv_channel_mean")
    return out


def se_mlp(pooled: Tensor, w1, b1, w2, b2) -> Tensor:
    n, c = pooled.shape
    cr = w1.shape[0]
    gate = torch.empty_like(pooled)
    w1, b1, w2, b2 = map(f32, (w1, b1, w2, b2))
    hidden = torch.empty((n, cr), device=pooled.device, dtype=torch.float32) if n <= 4 else None
    check(L.lib().hv_se_mlp2(pooled.data_ptr(), n, c, cr, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                             b2.data_ptr(), ptr(hidden), gate.data_ptr(), stream_ptr()), "hv_se_mlp2")
    return gate


def se_gate(x: Tensor, w1, b1, w2, b2) -> Tensor:
    """SE gate fp32 [n, c] of an NHWC map in one call (hv_se_gate): bitwise
    se_mlp(channel_mean(x), ...)."""
    _contig(x, "x")
    n, c = x.shape[0], x.shape[-1]
    hw = x.numel() // (n * c)
    cr = w1.shape[0]
    w1, b1, w2, b2 = map(f32, (w1, b1, w2, b2))
    gate = torch.empty((n, c), device=x.device, dtype=torch.float32)
    work = torch.empty(L.lib().hv_channel_mean_work_floats(n, hw, c), device=x.device, dtype=torch.float32)
    hidden = torch.empty((n, cr), device=x.device, dtype=torch.float32) if n <= 4 else None
    check(L.lib().hv_se_gate(dtype_code(x.dtype), x.data_ptr(), n, hw, c, cr, w1.data_ptr(), b1.data_ptr(),
                             w2.data_ptr(), b2.data_ptr(), work.data_ptr(), ptr(hidden), gate.data_ptr(),
                             stream_ptr()), "hv_se_gate")
    return gate


def scale_residual(x: Tensor, gate: Tensor, identity: Optional[Tensor]) -> Tensor:
    _contig(x, "x")
    n, c = x.shape[0], x.shape[-1]
    hw = x.numel() // (n * c)
    if gate.shape != (n, c) or gate.dtype != torch.float32 or not gate.is_contiguous():
        raise ValueError("scale_residual: gate must be contiguous fp32 [n, c]")
    y = torch.empty_like(x)
    if identity is not None:
        _contig(identity, "identity")
        if identity.shape != x.shape or identity.dtype != x.dtype:
            raise ValueError("scale_residual: identity must match x")
    check(L.lib().hv_scale_residual(dtype_code(x.dtype), x.data_ptr(), gate.data_ptr(), ptr(identity), n, hw, c,
                                    y.data_ptr(), stream_ptr()), "hv_scale_residual")
    return y


def upsample_add(a: Tensor, b: Tensor) -> Tensor:
    n, h, w, c = a.shape
    hb, wb = b.shape[1], b.shape[2]
    if b.shape[0] != n or b.shape[3] != c or a.dtype != b.dtype:
        raise ValueError("upsample_add: batch/channel/dtype mismatch")
    y = torch.empty_like(a)
    check(L.lib().hv_upsample_add(dtype_code(a.dtype), _contig(a, "a").data_ptr(), _contig(b, "b").data_ptr(),
                                  n, h, w, c, hb, wb, y.data_ptr(), stream_ptr()), "hv_upsample_add")
    return y


def add_scaled(a: Tensor, b: Tensor, alpha: float) -> Tensor:
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError(f"add_scaled: {tuple(a.shape)}/{a.dtype} vs {tuple(b.shape)}/{b.dtype}")
    y = torch.empty_like(a)
    check(L.lib().hv_add_scaled(dtype_code(a.dtype), _contig(a, "a").data_ptr(), _contig(b, "b").data_ptr(),
                                a.numel(), alpha, y.data_ptr(), stream_ptr()), "hv_add_scaled")
    return y


def add_rowvec(x: Tensor, v: Tensor) -> Tensor:
    n, c = x.shape[0], x.shape[-1]
    p = x.numel() // (n * c)
    v = f32(v)
    if v.shape != (n, c):
        raise ValueError(f"add_rowvec: v {tuple(v.shape)} != {(n, c)}")
    y = torch.empty_like(x)
    check(L.lib().hv_add_rowvec(dtype_code(x.dtype), _contig(x, "x").data_ptr(), v.data_ptr(), n, p, c,
                                y.data_ptr(), stream_ptr()), "hv_add_rowvec")
    return y


def interp_linear(src: Tensor, lout: int) -> Tensor:
    """[L, D] fp32 -> [lout, D] (F.interpolate mode='linear', align_corners=False, on dim 0)."""
    src = f32(src)
    Ls, D = src.shape
    dst = torch.empty((lout, D), device=src.device, dtype=torch.float32)
    check(L.lib().hv_interp_linear(src.data_ptr(), Ls, D, lout, dst.data_ptr(), stream_ptr()), "hv_interp_linear")
    return dst


def vit_tokens(x: Tensor, cls: Tensor, pos: Tensor, scale: Tensor) -> Tensor:
    """x [n, t, d] -> RMSNorm(cat(cls, x) + pos) [n, t+1, d]."""
    n, t, d = x.shape
    cls, pos, scale = f32(cls), f32(pos), f32(scale)      # keep temporaries alive over the launch
    if cls.numel() != d or pos.shape != (t + 1, d) or scale.numel() != d:
        raise ValueError("vit_tokens: cls/pos/scale shape mismatch")
    y = torch.empty((n, t + 1, d), device=x.device, dtype=x.dtype)
    check(L.lib().hv_vit_tokens(dtype_code(x.dtype), _contig(x, "x").data_ptr(), cls.data_ptr(),
                                pos.data_ptr(), scale.data_ptr(), n, t, d, y.data_ptr(), stream_ptr()),
          "hv_vit_tokens")
    return y


def attention(q: Tensor, k: Tensor, v: Tensor, heads: int) -> Tensor:
    n, Lq, D = q.shape
    hd = D // heads
    o = torch.empty_like(q)
    if q.dtype == torch.bfloat16 and hd == 32:
        vt = torch.empty(L.lib().hv_attention_work_elems(n, Lq, heads, hd), device=q.device, dtype=q.dtype)
        check(L.lib().hv_attention_mfma(_contig(q, "q").data_ptr(), _contig(k, "k").data_ptr(),
                                        _contig(v, "v").data_ptr(), vt.data_ptr(), o.data_ptr(), n, Lq, heads, hd,
                                        hd ** -0.5, stream_ptr()), "hv_attention_mfma")
        return o
    check(L.lib().hv_attention(dtype_code(q.dtype), _contig(q, "q").data_ptr(), _contig(k, "k").data_ptr(),
                               _contig(v, "v").data_ptr(), o.data_ptr(), n, Lq, heads, hd, hd ** -0.5,
                               stream_ptr()), "hv_attention")
    return o


def attention_general(q: Tensor, k: Tensor, v: Tensor, heads: int, key_padding_mask: Optional[Tensor] = None,
                      need_weights: bool = False):
    """softmax(q k^T / sqrt(hd), masked) v for q [n, Lq, D], k / v [n, Lk, D] -> (out [n, Lq, D],
    weights [n, heads, Lq, Lk] fp32 or None).  key_padding_mask: bool [n, Lk], True = ignore."""
    n, Lq, D = q.shape
    Lk = k.shape[1]
    if k.shape != (n, Lk, D) or v.shape != k.shape or k.dtype != q.dtype or v.dtype != q.dtype:
        raise ValueError("attention_general: q/k/v shapes or dtypes disagree")
    hd = D // heads
    mask = None
    if key_padding_mask is not None:
        if tuple(key_padding_mask.shape) != (n, Lk):
            raise ValueError(f"key_padding_mask must be [{n}, {Lk}]")
        mask = key_padding_mask.to(device=q.device, dtype=torch.uint8).contiguous()
    o = torch.empty_like(q)
    w = torch.empty((n, heads, Lq, Lk), device=q.device, dtype=torch.float32) if need_weights else None
    check(L.lib().hv_attention_general(dtype_code(q.dtype), _contig(q, "q").data_ptr(), _contig(k, "k").data_ptr(),
                                       _contig(v, "v").data_ptr(), ptr(mask), o.data_ptr(), ptr(w), n, Lq, Lk,
                                       heads, hd, hd ** -0.5, stream_ptr()), "hv_attention_general")
    return o, w


def gather_rows(x: Tensor, stride_rows: int) -> Tensor:
    """Row 0 of every group of `stride_rows` rows: x [n*stride_rows, c] -> [n, c]."""
    c = x.shape[-1]
    rows = x.numel() // c
    if rows % stride_rows:
        raise ValueError("gather_rows: row count is not a multiple of stride_rows")
    n = rows // stride_rows
    y = torch.empty((n, c), device=x.device, dtype=x.dtype)
    check(L.lib().hv_gather_rows(dtype_code(x.dtype), _contig(x, "x").data_ptr(), stride_rows, n, c,
                                 y.data_ptr(), stream_ptr()), "hv_gather_rows")
    return y


def yolo_decode(logits: Tensor, A: int, nc: int, anchor_wh: Tensor, detections: bool = False):
    """logits NHWC [n, h, w, A*(5+nc)] -> reference YOLODecoder outputs (shim S5 layout); with
    detections=True the dict also holds 'detections' [n, A, h, w, 5+nc] = (xyxy box,
    objectness, class probabilities), written by the same launch."""
    n, h, w, _ = logits.shape
    dev = logits.device
    P = 5 + nc
    pred = torch.empty((n, A, h, w, P), device=dev, dtype=torch.float32)
    boxes = torch.empty((n, A, h, w, 4), device=dev, dtype=torch.float32)
    scores = torch.empty((n, A, h, w, nc), device=dev, dtype=torch.float32)
    cs = torch.empty((n, A, h, w), device=dev, dtype=torch.float32)
    ci = torch.empty((n, A, h, w), device=dev, dtype=torch.int64)
    obj = torch.empty((n, A, h, w, 1), device=dev, dtype=torch.float32)
    det = torch.empty((n, A, h, w, P), device=dev, dtype=torch.float32) if detections else None
    awh = f32(anchor_wh)
    if awh.numel() != 2 * A or logits.shape[-1] != A * P:
        raise ValueError("yolo_decode: anchor / channel count mismatch")
    check(L.lib().hv_yolo_decode(dtype_code(logits.dtype), _contig(logits, "logits").data_ptr(), n, h, w, A, nc,
                                 awh.data_ptr(), pred.data_ptr(), boxes.data_ptr(), scores.data_ptr(),
                                 cs.data_ptr(), ci.data_ptr(), obj.data_ptr(), ptr(det), stream_ptr()),
          "hv_yolo_decode")
    out = {"boxes": boxes, "scores": scores, "class_scores": cs, "class_indices": ci,
           "objectness": obj, "raw_predictions": pred}
    if det is not None:
        out["detections"] = det
    return out, pred


def _dense(t: Tensor) -> bool:
    """Non-overlapping and dense (a permutation of a contiguous layout, e.g. the NCHW views
    of NHWC storage): its bytes are one range starting at data_ptr()."""
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def clone_tree(tree):
    """Owned copies of every device tensor in a (nested dict / list / tuple) output tree:
    one arena allocation + one hv_copy_segments launch per 64 tensors, same shapes, strides
    and dtypes (a graph replay's static outputs, handed to callers that keep them)."""
    leaves = []

    def collect(o):
        if isinstance(o, Tensor):
            leaves.append(o)
        elif isinstance(o, dict):
            for v in o.values():
                collect(v)
        elif isinstance(o, (list, tuple)):
            for v in o:
                collect(v)
    collect(tree)
    uniq = {}
    for t in leaves:
        if t.is_cuda and id(t) not in uniq:
            uniq[id(t)] = t if _dense(t) else t.contiguous()
    if not uniq:
        return tree
    offs, total = {}, 0
    for k, t in uniq.items():
        offs[k] = total
        total += (t.numel() * t.element_size() + 255) // 256 * 256
    dev = next(iter(uniq.values())).device
    arena = torch.empty(max(total, 1), device=dev, dtype=torch.uint8)
    segs = (L.CopySegment * len(uniq))()
    new = {}
    for i, (k, t) in enumerate(uniq.items()):
        nb = t.numel() * t.element_size()
        flat = arena[offs[k]:offs[k] + nb].view(t.dtype)
        d = torch.as_strided(flat, t.shape, t.stride())
        new[k] = d
        segs[i].src, segs[i].dst, segs[i].bytes = t.data_ptr(), d.data_ptr(), nb
    check(L.lib().hv_copy_segments(segs, len(uniq), stream_ptr()), "hv_copy_segments")

    def rebuild(o):
        if isinstance(o, Tensor):
            return new.get(id(o), o)
        if isinstance(o, dict):
            return {k: rebuild(v) for k, v in o.items()}
        if isinstance(o, list):
            return [rebuild(v) for v in o]
        if isinstance(o, tuple):
            return tuple(rebuild(v) for v in o)
        return o
    return rebuild(tree)


# ---------------------------------------------------------------------------- post-processing
class NmsPlan:
    """GPU post_process (hv_nms) over a FIXED set of decoded tensors: the device table and the
    output / work buffers are built once, so run() is two kernel launches with no host work --
    capturable inside a hipGraph (the streaming pipeline records it after the forward).
    decoded: {scale_key: {'boxes' [B,A,H,W,4], 'class_scores' [B,A,H,W], 'class_indices'}}."""

    def __init__(self, decoded, conf_thr: float, iou_thr: float, max_det: int):
        keys = sorted(decoded)
        ents = (L.NmsScale * len(keys))()
        self._keep = []
        B = dev = None
        for i, k in enumerate(keys):
            o = decoded[k]
            bx, sc, ci = o["boxes"], o["class_scores"], o["class_indices"]
            if bx.dtype != torch.float32 or sc.dtype != torch.float32 or ci.dtype != torch.int64 or \
                    not (bx.is_contiguous() and sc.is_contiguous() and ci.is_contiguous()):
                bx = bx.detach().float().contiguous()
                sc = sc.detach().float().contiguous()
                ci = ci.detach().to(torch.int64).contiguous()
            _cuda(bx, sc, ci)
            B = sc.shape[0]
            dev = sc.device
            cells = sc.numel() // B
            if bx.numel() != B * cells * 4 or ci.numel() != B * cells:
                raise ValueError("nms: boxes / scores / indices shapes disagree")
            ents[i].boxes, ents[i].class_scores, ents[i].class_indices, ents[i].cells = \
                bx.data_ptr(), sc.data_ptr(), ci.data_ptr(), cells
            self._keep += [bx, sc, ci]
        self.table = tables.upload(ents, dev, self, "scales")
        self.n_scales, self.B = len(keys), B
        self.conf, self.iou, self.max_det = float(conf_thr), float(iou_thr), int(max_det)
        self.boxes = torch.empty((B, max_det, 4), device=dev, dtype=torch.float32)
        self.scores = torch.empty((B, max_det), device=dev, dtype=torch.float32)
        self.labels = torch.empty((B, max_det), device=dev, dtype=torch.int64)
        self.count = torch.empty(B, device=dev, dtype=torch.int32)
        if int(max_det) < 1:
            raise ValueError("nms: max_det must be >= 1")
        self.max_cells = max(int(o["class_scores"].numel()) // B for o in decoded.values())
        nbytes = L.lib().hv_nms_work_bytes(B, len(keys), self.max_det, self.max_cells)
        if nbytes == 0:
            raise ValueError(f"nms: unsupported sizes (batch {B}, max_det {max_det}, cells {self.max_cells})")
        self.work = torch.empty(nbytes, device=dev, dtype=torch.uint8)

    def run(self):
        check(L.lib().hv_nms(self.table.data_ptr(), self.n_scales, self.B, self.conf, self.iou, self.max_det,
                             self.max_cells, self.boxes.data_ptr(), self.scores.data_ptr(), self.labels.data_ptr(),
                             self.count.data_ptr(), self.work.data_ptr(), stream_ptr()), "hv_nms")
        return self.boxes, self.scores, self.labels, self.count


def sort_desc_exact(vals: torch.Tensor, depth_limit: int = -1) -> torch.Tensor:
    """torch.sort(vals, descending=True).indices of the reference's CPU sort (libstdc++ introsort,
    tie order included), on the GPU (hv_sort_desc_exact; the sort hv_nms falls back to on ties).
    depth_limit >= 0 forces introsort's depth limit (reaches its heap-sort fallback)."""
    v = vals.detach().float().contiguous().reshape(-1)
    _cuda(v)
    n = v.numel()
    out = torch.empty(n, device=v.device, dtype=torch.int32)
    if n == 0:
        return out.long()
    work = torch.empty(L.lib().hv_sort_desc_exact_work_bytes(n), device=v.device, dtype=torch.uint8)
    check(L.lib().hv_sort_desc_exact(v.data_ptr(), n, int(depth_limit), out.data_ptr(), work.data_ptr(),
                                     stream_ptr()), "hv_sort_desc_exact")
    return out.long()


def nms_batched(decoded, conf_thr: float, iou_thr: float, max_det: int):
    """GPU post_process (hv_nms): per-scale threshold + greedy NMS, then cross-scale NMS.
    Returns device tensors boxes [B, max_det, 4], scores [B, max_det], labels [B, max_det],
    count [B] (int32)."""
    return NmsPlan(decoded, conf_thr, iou_thr, max_det).run()


# ---------------------------------------------------------------------------- preprocessing
IMAGENET_MEAN_STD = (0.485, 0.456, 0.406, 0.229, 0.224, 0.225)


_PIL_TABLES = {}


def pil_table(h: int, w: int, height: int, width: int, device) -> Tensor:
    """Device copy of the Pillow-exact resample table for (h, w) -> (height, width), cached."""
    key = (h, w, height, width, str(device))
    t = _PIL_TABLES.get(key)
    if t is None:
        n = L.lib().hv_pil_table_ints(h, w, height, width)
        host = torch.empty(n, dtype=torch.int32)
        check(L.lib().hv_pil_resample_tables(h, w, height, width, host.data_ptr()), "hv_pil_resample_tables")
        t = host.to(device)
        _PIL_TABLES[key] = t
    return t


def preprocess(frames: Tensor, height: int, width: int, *, bgr: bool = True, dtype: torch.dtype = torch.float32,
               nhwc: bool = False, mean_std=IMAGENET_MEAN_STD, resample: str = "pil",
               out: Optional[Tensor] = None) -> Tensor:
    """uint8 [n, h, w, 3] device frames -> normalised [n, 3, height, width] (NCHW tensor, or the
    NCHW-shaped view of NHWC storage when nhwc=True -- zero-copy for the model's input).
    resample: 'pil' (the reference's torchvision/Pillow path, bit-exact) or 'bilinear'
    (F.interpolate / kornia semantics).  `out` (contiguous, the NHWC or NCHW buffer) is written
    in place when given (the streaming pipeline's captured input)."""
    _cuda(frames)
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError("preprocess expects uint8 [n, h, w, 3] frames")
    frames = frames.contiguous()
    n, h, w, _ = frames.shape
    code = {torch.float32: L.HV_F32, torch.bfloat16: L.HV_BF16, torch.float16: 2}[dtype]
    shape = (n, height, width, 3) if nhwc else (n, 3, height, width)
    if out is None:
        out = torch.empty(shape, device=frames.device, dtype=dtype)
    elif tuple(out.shape) != shape or out.dtype != dtype or not out.is_contiguous():
        raise ValueError(f"preprocess: out must be a contiguous {dtype} {shape} tensor")
    ms = (C.c_float * 6)(*mean_std)
    if resample == "pil":
        tab = pil_table(h, w, height, width, frames.device)
        check(L.lib().hv_preprocess_pil(frames.data_ptr(), n, h, w, int(bgr), height, width, tab.data_ptr(), ms,
                                        code, int(nhwc), out.data_ptr(), stream_ptr()), "hv_preprocess_pil")
    elif resample == "bilinear":
        check(L.lib().hv_preprocess(frames.data_ptr(), n, h, w, int(bgr), height, width, ms, code, int(nhwc),
                                    out.data_ptr(), stream_ptr()), "hv_preprocess")
    else:
        raise ValueError("resample must be 'pil' or 'bilinear'")
    return out.permute(0, 3, 1, 2) if nhwc else out


# ---------------------------------------------------------------------------- stability monitor
def symeig_group(mats, outs=None) -> list:
    """Ascending eigenvalues of (H + H^T)/2 for every square fp32 matrix in `mats`, all in one
    grouped launch sequence (hv_symeig_group) -- the eigvalsh of _monitor_stability
    (manifold_layers.py:288-290).  `outs` (fp32 [n] each) are written in place when given."""
    mats = [_contig(m.detach(), "H") for m in mats]
    if not mats:
        return []
    _cuda(*mats)
    for m in mats:
        if m.dim() != 2 or m.shape[0] != m.shape[1] or m.dtype != torch.float32:
            raise ValueError("symeig_group: square fp32 matrices")
    dev = mats[0].device
    if outs is None:
        outs = [torch.empty(m.shape[0], device=dev, dtype=torch.float32) for m in mats]
    lib = L.lib()
    order = sorted(range(len(mats)), key=lambda i: -mats[i].shape[0])
    entries = (L.SymeigEntry * len(mats))()
    ns = (C.c_int * len(mats))()
    works, rs = [], 0
    for k, i in enumerate(order):
        n = mats[i].shape[0]
        if outs[i].numel() != n or outs[i].dtype != torch.float32 or not outs[i].is_contiguous():
            raise ValueError("symeig_group: outputs must be contiguous fp32 [n]")
        w = torch.empty(lib.hv_symeig_work_doubles(n), device=dev, dtype=torch.float64)
        works.append(w)
        e = entries[k]
        e.h, e.eig, e.work, e.n, e.row_start = mats[i].data_ptr(), outs[i].data_ptr(), w.data_ptr(), n, rs
        ns[k] = n
        rs += n
    table = upload_table(entries, dev)
    check(lib.hv_symeig_group(table.data_ptr(), ns, len(mats), stream_ptr()), "hv_symeig_group")
    return outs


def stability_stats(x_in: Tensor, x_out: Tensor, h: Tensor, history: Optional[Tensor] = None,
                    slot: int = 0) -> Tensor:
    """[signal_ratio, row_sum_error, col_sum_error] (manifold_layers.py:296-315) as a device
    fp32 [3]; history[slot] = signal_ratio when `history` is given (:300-303)."""
    D = x_in.shape[-1]
    xi = _contig(x_in.detach(), "x_in").reshape(-1, D)
    xo = _contig(x_out.detach(), "x_out").reshape(-1, D)
    if xo.dtype != xi.dtype:
        xo = xo.to(xi.dtype)
    hh = _contig(h.detach().float(), "H")
    _cuda(xi, xo, hh)
    lib = L.lib()
    work = torch.empty(lib.hv_stability_work_floats(xi.shape[0]), device=xi.device, dtype=torch.float32)
    out = torch.empty(3, device=xi.device, dtype=torch.float32)
    check(lib.hv_stability_stats(dtype_code(xi.dtype), xi.data_ptr(), xo.data_ptr(), xi.shape[0], D,
                                 hh.data_ptr(), hh.shape[0], work.data_ptr(), ptr(history), slot,
                                 out.data_ptr(), stream_ptr()), "hv_stability_stats")
    return out


# ---------------------------------------------------------------------------- diagnostics
KERNEL_FAMILIES = ("gemm_pp256", "glds_128x128", "glds_64x128", "glds_128x64", "glds_64x64", "gemm_regstage",
                   "mhc_fused", "attn_mfma", "attn_scalar", "sinkhorn_group", "attn_general", "gemm_smallk",
                   "gemm_splitk")


def launch_counts(reset: bool = False) -> dict:
    """Host-side launch counts per kernel family since the last reset (include/hv_tuning.h)."""
    arr = (C.c_longlong * 16)()
    L.lib().hv_diag_launch_counts(arr)
    if reset:
        L.lib().hv_diag_reset_counts()
    return {n: int(arr[i]) for i, n in enumerate(KERNEL_FAMILIES)}


# ---------------------------------------------------------------------------- debug tracing
def _install_sync_check():
    """HV_SYNC_CHECK=1: synchronise after every op and report the first one that faults."""
    import functools
    import os
    import sys
    if os.environ.get("HV_SYNC_CHECK") != "1":
        return
    mod = sys.modules[__name__]
    for name in ("gemm", "conv2d", "conv_weight_prep", "bn_fold", "cast", "row_stats", "layernorm", "rmsnorm",
                 "sinkhorn", "mhc_prep", "nchw_to_nhwc", "maxpool2x2", "channel_mean", "se_mlp", "se_gate",
                 "scale_residual", "upsample_add", "add_scaled", "add_rowvec", "interp_linear", "vit_tokens",
                 "attention", "gather_rows", "yolo_decode"):
        fn = getattr(mod, name)

        def wrap(fn=fn, name=name):
            @functools.wraps(fn)
            def inner(*a, **k):
                desc = [tuple(t.shape) if isinstance(t, torch.Tensor) else t for t in a]
                print(f"[hv] {name} {desc}", flush=True)
                r = fn(*a, **k)
                torch.cuda.synchronize()
                return r
            return inner
        setattr(mod, name, wrap())
    run0 = SinkhornGroup.run

    def run(self, raws=None):
        print(f"[hv] sinkhorn_group n={len(self.entries)} totals={self.totals}", flush=True)
        r = run0(self, raws)
        torch.cuda.synchronize()
        return r
    SinkhornGroup.run = run


_install_sync_check()
