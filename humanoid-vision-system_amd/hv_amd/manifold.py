"""mHC layers on the HIP path: Sinkhorn projection, ManifoldHyperConnection, mHC attention,
RMSNorm.  Parameter/buffer names and shapes mirror reference src/models/manifold_layers.py so
reference checkpoints load unchanged.

mHC forward (manifold_layers.py:223-280), eval mode, restated for MI355X:
    z   = (x - mean) * rstd                                   LayerNorm core, applied on load
    h1  = GELU(z A1 + c1)      A1 = Gc W1^T, c1 = u W1^T + b1  (folded; or z Gc + u, then W1)
    h2  = GELU(h1 W2^T + b2)
    yc  = [x | h2] Wc          Wc = [H_res - rowmean ; H_post - rowmean]
    out = LN_post(yc)
with G = diag(gamma_pre) sigmoid(H_pre_raw), Gc = G - colmean_i(G), u = beta_pre sigmoid(H_pre_raw).
Centering is exact because LayerNorm subtracts the row mean (sum_i z_i = 0; LN_post(y) =
LN_post(y - const_row)); it removes the ~1/D-uniform part of H_res and the ~1.0-uniform part
of H_post, which is what makes the reference's bf16 path O(1)-wrong.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, Dict, Optional

import torch
import torch.nn as nn

from . import ops
from .runtime import RunCtx, current, module_options, options, require_cuda, resolve_dtype, use_ctx


# ================================================================== stability monitor queue
# (H_res, eigenvalues buffer) of every _monitor_stability call since the last flush, keyed by the
# buffer (a site monitored twice keeps its latest matrix): solved together by one grouped
# hv_symeig_group -- 2*(max n - 2) + 3 launches for all 76 sites instead of per site.
_EIG_QUEUE: Dict[int, Any] = {}


def queue_eigvals(h: torch.Tensor, out: torch.Tensor) -> None:
    _EIG_QUEUE[id(out)] = (h, out)
    if len(_EIG_QUEUE) >= 512:
        flush_stability()


def flush_stability() -> None:
    """Solve every queued eigenvalue problem (manifold_layers.py:288-290) in one launch group."""
    if not _EIG_QUEUE:
        return
    items = list(_EIG_QUEUE.values())
    _EIG_QUEUE.clear()
    ops.symeig_group([h for h, _ in items], [o for _, o in items])


# ================================================================== Sinkhorn
class SinkhornKnoppProjection(nn.Module):
    """Reference manifold_layers.py:10-101 (shim S1: 2-D input = batch of one)."""

    def __init__(self, num_iterations: int = 20, epsilon: float = 1e-8, tau: float = 1.0):
        super().__init__()
        self.num_iterations = num_iterations
        self.epsilon = epsilon
        self.tau = tau
        self.register_buffer("convergence_history", torch.zeros(num_iterations))

    def forward(self, matrix: torch.Tensor, return_history: bool = False):
        require_cuda(matrix, "SinkhornKnoppProjection")
        g = ops.SinkhornGroup([matrix.detach().float().contiguous()], [self.num_iterations],
                              matrix.device, self.epsilon, self.tau)
        if matrix.requires_grad and torch.is_grad_enabled():
            # autograd through every iteration (grouped reverse sweep, hv_sinkhorn_group_backward)
            from .train_fn import SinkhornGroupFn
            if matrix.dtype != torch.float32 or not matrix.is_contiguous():
                raise TypeError("SinkhornKnoppProjection: differentiable input must be contiguous fp32")
            (out,) = SinkhornGroupFn.apply(g, None, matrix)
        else:
            out = g.run()[0]
            out = out.squeeze(0) if matrix.dim() == 2 else out
        self.convergence_history.copy_(g.hists[0][: self.num_iterations])
        if not return_history:
            return out
        return out, self._history_dict(g)

    def _history_dict(self, g: "ops.SinkhornGroup") -> Dict[str, Any]:
        # reference :86-91: per-iteration means of the row sums and of the column sums
        e = g.entries[0]
        b, n, m, it = e.batch, e.n, e.m, e.iters
        w = g.works[0]
        a_sz, b_sz = (it + 1) * b * n, (it + 1) * b * m
        bh = w[a_sz:a_sz + b_sz].view(it + 1, b * m)
        rh = w[a_sz + b_sz:a_sz + b_sz + it * b * n].view(it, b * n)
        cs = (bh[:-1] / bh[1:] - self.epsilon)
        rows = rh.mean(dim=1).tolist()
        cols = cs.mean(dim=1).tolist()
        return {"row_sums": rows, "col_sums": cols, "final_row_error": rows[-1] - 1.0,
                "final_col_error": cols[-1] - 1.0}

    def get_convergence_metrics(self) -> Dict[str, Any]:
        h = self.convergence_history
        return {"mean_convergence": h.mean().item(), "max_convergence": h.max().item(),
                "final_convergence": h[-1].item()}


# ================================================================== mHC plan
# HVOptions.fold_max_d (default 1024): fold H_pre into W1 for every site but the D=1792 final
# fusion; HVOptions.use_fused_mhc: one-launch kernel for the small-D sites (hv_mhc_fused)


@dataclass
class MhcPlan:
    D: int
    Hd: int
    fold: bool
    dtype: torch.dtype
    b1: torch.Tensor          # fold: a1t [2Hd, D]; else gct [Hd, D]
    c1: torch.Tensor          # fold: c1 [2Hd] fp32; else u [Hd] fp32
    w1: Optional[torch.Tensor]
    bias1: Optional[torch.Tensor]
    w2: torch.Tensor
    bias2: torch.Tensor
    wct: torch.Tensor
    g_post: torch.Tensor
    b_post: torch.Tensor
    cs: Optional[torch.Tensor] = None   # row sums of b1 as stored: LayerNorm applied after GEMM1


def build_plan(m: "ManifoldHyperConnection", h_res: torch.Tensor, dtype: torch.dtype,
               fold_max_d: int = 1024) -> MhcPlan:
    """Per-site coefficient prep (about ten launches per site).  The forward uses the grouped
    prep.PrepProgram; this path is kept as its independent cross-check (tests/test_gpu_prep.py)."""
    D, Hd = m.input_dim, m.hidden_dim
    fold = D <= fold_max_d and Hd % 32 == 0
    gc, u, wct = ops.mhc_prep(m.H_pre_raw, m.H_post_raw, h_res, m.norm_pre.weight, m.norm_pre.bias,
                              gc_transposed=not fold)
    w1 = ops.f32(m.mlp[0].weight)
    b1 = ops.f32(m.mlp[0].bias)
    if fold:
        # A1^T = W1 Gc^T  [2Hd, D];  c1 = W1 u + b1
        a1t = ops.gemm(ops.cast(w1, dtype), ops.cast(gc, dtype), out_dtype=dtype)
        c1 = ops.gemv(w1, u, b1)
        first, second, w1c, b1c = a1t, c1, None, None
    else:
        first, second, w1c, b1c = ops.cast(gc, dtype), u, ops.cast(w1, dtype), b1
    return MhcPlan(D=D, Hd=Hd, fold=fold, dtype=dtype, b1=first, c1=second, w1=w1c, bias1=b1c,
                   w2=ops.cast(ops.f32(m.mlp[3].weight), dtype), bias2=ops.f32(m.mlp[3].bias),
                   wct=ops.cast(wct, dtype), g_post=ops.f32(m.norm_post.weight),
                   b_post=ops.f32(m.norm_post.bias))


def mhc_apply(x2: torch.Tensor, p: MhcPlan, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Token chain on x2 [T, D] (compute dtype).  Returns LN_post(...) (+ residual) [T, D]."""
    if (options().use_fused_mhc and p.fold and x2.is_contiguous()
            and ops.mhc_fused_supported(p.D, p.Hd, x2.dtype, T=x2.shape[0])
            and (residual is None or residual.dtype == x2.dtype)):
        return ops.mhc_fused(x2, p.b1, p.c1, p.w2, p.bias2, p.wct, p.g_post, p.b_post, residual)
    mean, rstd = ops.row_stats(x2, 1e-5)
    if p.fold:
        h1 = ops.gemm(x2, p.b1, bias=p.c1, act="gelu", a_mean=mean, a_rstd=rstd, b_colsum=p.cs)
    else:
        e = ops.gemm(x2, p.b1, bias=p.c1, a_mean=mean, a_rstd=rstd, b_colsum=p.cs)
        h1 = ops.gemm(e, p.w1, bias=p.bias1, act="gelu")
    h2 = ops.gemm(h1, p.w2, bias=p.bias2, act="gelu")
    yc = ops.gemm(x2, p.wct, a2=h2, out_dtype=torch.float32)
    return ops.layernorm(yc, p.g_post, p.b_post, 1e-5, out_dtype=x2.dtype, residual=residual)


def prepare_plans(mods, ctx: RunCtx, cache: Optional[dict] = None, key=None, overlap: bool = False,
                  groups: Optional[dict] = None) -> None:
    """Sinkhorn + coefficient prep for every mHC module in `mods` through one grouped
    PrepProgram (reused from `cache` while `key` -- the owner's parameter/buffer storage --
    and the precision are unchanged, so a captured graph replays the same buffers)."""
    from .prep import PrepProgram
    mods = [m for m in mods if id(m) not in ctx.plans]
    if not mods:
        return
    prog = None
    fmd = ctx.opts.fold_max_d
    if cache is not None and cache.get("key") == (key, ctx.dtype, fmd):
        prog = cache["program"]
    if prog is None:
        prog = PrepProgram(mods, ctx.dtype, mods[0].H_res_raw.device, fmd, groups)
        if cache is not None:
            cache["key"], cache["program"] = (key, ctx.dtype, fmd), prog
    ctx.program = prog
    prog.run(ctx, overlap)


# ================================================================== mHC layer
class ManifoldHyperConnection(nn.Module):
    """Reference manifold_layers.py:104-346 (same parameters, buffers and init)."""

    def __init__(self, input_dim: int, expansion_rate: int = 4, hidden_dim: Optional[int] = None,
                 alpha: float = 0.01, sk_iterations: int = 20, use_mixed_precision: bool = True,
                 dropout_rate: float = 0.1):
        super().__init__()
        self.input_dim = input_dim
        self.expansion_rate = expansion_rate
        self.hidden_dim = hidden_dim or input_dim * expansion_rate
        self.alpha = alpha
        self.use_mixed_precision = use_mixed_precision
        self.dropout_rate = dropout_rate
        D, Hd = input_dim, self.hidden_dim
        # torch.randn * alpha first (manifold_layers.py:149-157): the Xavier re-init below
        # overwrites the values, but the draws keep a seeded model's RNG stream the reference's
        self.H_pre_raw = nn.Parameter(torch.randn(D, Hd) * alpha)
        self.H_post_raw = nn.Parameter(torch.randn(Hd, D) * alpha)
        self.H_res_raw = nn.Parameter(torch.randn(D, D) * alpha)
        self.sinkhorn = SinkhornKnoppProjection(sk_iterations)
        self.mlp = nn.Sequential(nn.Linear(Hd, 2 * Hd), nn.GELU(), nn.Dropout(dropout_rate),
                                 nn.Linear(2 * Hd, Hd), nn.GELU(), nn.Dropout(dropout_rate))
        self.norm_pre = nn.LayerNorm(D)
        self.norm_post = nn.LayerNorm(D)
        self.dropout = nn.Dropout(dropout_rate)
        self.register_buffer("gradient_norms", torch.zeros(3))
        self.register_buffer("eigenvalues", torch.zeros(D))
        self.register_buffer("signal_ratio_history", torch.zeros(1000))
        self.signal_ratio_idx = 0
        self.hv_precision = "bf16" if use_mixed_precision else "fp32"
        self._frozen = None
        for p in (self.H_pre_raw, self.H_post_raw, self.H_res_raw):   # :194-196
            nn.init.xavier_uniform_(p, gain=0.1)
        for lyr in (self.mlp[0], self.mlp[3]):                         # :199-203
            nn.init.xavier_uniform_(lyr.weight, gain=math.sqrt(2))
            nn.init.zeros_(lyr.bias)
        # the eigenvalue solves queued by monitor_stability land before anyone reads the
        # buffers through state_dict() / checkpoints (the reference writes them every forward)
        self.register_state_dict_pre_hook(lambda *_a, **_k: flush_stability())

    @property
    def dtype(self):
        return torch.bfloat16 if self.use_mixed_precision else torch.float32

    def constrained_matrices(self):
        """(H_pre, H_post, H_res) (manifold_layers.py:205-221); the Sinkhorn runs on the GPU."""
        require_cuda(self.H_res_raw, "constrained_matrices")
        H_pre = torch.sigmoid(self.H_pre_raw)
        H_post = 2 * torch.sigmoid(self.H_post_raw)
        H_res = self.sinkhorn(self.H_res_raw)
        return H_pre, H_post, H_res

    def plan(self) -> MhcPlan:
        ctx = current()
        if ctx is not None:
            ctx.join_prep()
            p = ctx.plans.get(id(self))
            if p is None:
                prepare_plans([self], ctx)
                p = ctx.plans[id(self)]
            return p
        own = RunCtx(dtype=resolve_dtype(self), opts=module_options(self))
        prepare_plans([self], own)
        return own.plans[id(self)]

    def forward_tokens(self, x2: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x2: [T, D] token-major in the compute dtype."""
        if self.training:
            from . import train_fn as TF
            y = TF.mhc(self, x2, self.sinkhorn(self.H_res_raw))
            return y if residual is None else TF.AddFn.apply(y, residual, 1.0)
        return mhc_apply(x2, self.plan(), residual)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        require_cuda(x, "ManifoldHyperConnection")
        shape = x.shape
        dt = resolve_dtype(self)
        x2 = x.reshape(-1, shape[-1])
        in_dtype = x2.dtype
        x2 = x2.to(dt).contiguous()
        y = self.forward_tokens(x2)
        return y.view(shape).to(in_dtype if in_dtype in (torch.float32, torch.bfloat16) else dt)

    monitor_every = 1      # training-mode stability monitor period (reference: every forward)

    @torch.no_grad()
    def monitor_stability(self, H_res: torch.Tensor, x_in: torch.Tensor, x_out: torch.Tensor) -> None:
        """_monitor_stability (manifold_layers.py:282-316) on the device, no .item() in the
        training forward: the signal-growth ratio (into the circular history) and the row/column
        sum errors come from hv_stability_stats now; the eigenvalues of (H_res + H_res^T)/2 are
        queued and solved for every queued site at once (hv_symeig_group) at the end of the
        training forward or on the first metrics read (flush_stability)."""
        h = H_res.detach().float().contiguous()
        queue_eigvals(h, self.eigenvalues)
        slot = self.signal_ratio_idx % 1000
        st = ops.stability_stats(x_in, x_out, h, self.signal_ratio_history, slot)
        self.signal_ratio_idx += 1
        self._monitor_dev = {"signal_ratio": st[0], "row_sum_error": st[1], "col_sum_error": st[2]}

    @property
    def monitoring_metrics(self) -> Dict[str, float]:
        d = getattr(self, "_monitor_dev", None)
        if d is None:
            raise AttributeError("monitoring_metrics")
        flush_stability()
        ev = self.eigenvalues
        out = {"max_eigenvalue": ev.max().item(), "min_eigenvalue": ev.min().item()}
        out.update({k: float(v) for k, v in d.items()})
        return out

    def get_stability_metrics(self) -> Dict[str, Any]:
        """manifold_layers.py:318-341 (host reads happen here, never in forward)."""
        flush_stability()
        ev = self.eigenvalues
        metrics = {"max_eigenvalue": ev.max().item(), "min_eigenvalue": ev.min().item(),
                   "eigenvalue_range": (ev.max() - ev.min()).item(),
                   "sk_convergence": self.sinkhorn.get_convergence_metrics()}
        if self.signal_ratio_idx > 0:
            h = self.signal_ratio_history[: min(self.signal_ratio_idx, 1000)]
            metrics.update({"signal_ratio_mean": h.mean().item(), "signal_ratio_std": h.std().item(),
                            "signal_ratio_min": h.min().item(), "signal_ratio_max": h.max().item()})
        if getattr(self, "_monitor_dev", None) is not None:
            metrics.update(self.monitoring_metrics)
        return metrics

    def extra_repr(self) -> str:
        return (f"input_dim={self.input_dim}, hidden_dim={self.hidden_dim}, "
                f"expansion={self.expansion_rate}, alpha={self.alpha}")


# ================================================================== attention / norms
# HVOptions.parallel_qkv: q / k / v on three streams -- measured slower (22.30 vs 21.77 ms,
# tools/ab_vit.py); HVOptions.group_qkv: q / k / v GEMM1 as one N = 3*2Hd GEMM (shared LN stats)


class MultiHeadManifoldAttention(nn.Module):
    """Reference manifold_layers.py:349-434: four mHC projections around softmax(QK^T/sqrt(hd))V."""

    def __init__(self, embed_dim: int, num_heads: int = 8, dropout: float = 0.1, use_mhc: bool = True,
                 sk_iterations: int = 20):
        super().__init__()
        assert embed_dim % num_heads == 0
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.use_mhc = use_mhc
        if not use_mhc:
            raise NotImplementedError("hv_amd implements the use_mhc=True attention (the reference default)")
        kw = dict(expansion_rate=2, sk_iterations=sk_iterations)
        self.q_proj = ManifoldHyperConnection(embed_dim, **kw)
        self.k_proj = ManifoldHyperConnection(embed_dim, **kw)
        self.v_proj = ManifoldHyperConnection(embed_dim, **kw)
        self.out_proj = ManifoldHyperConnection(embed_dim, **kw)
        self.dropout = nn.Dropout(dropout)
        self.scaling = self.head_dim ** -0.5
        self._side = None

    def forward_tokens(self, x: torch.Tensor, n: int) -> torch.Tensor:
        """Self-attention on x [n*L, D] (compute dtype); returns out_proj(attn) [n*L, D].
        The q / k / v projections are independent mHC chains of small-M GEMMs (M = n*L, K =
        256): with HVOptions.parallel_qkv they run on three streams (three branches of a captured
        graph), so their latency-bound launches overlap."""
        L = x.shape[0] // n
        ctx = current()
        opts = options()
        if opts.use_fused_mhc and not self.training:
            # q / k / v read the same x: one grouped launch of the token-tile fused kernel
            qp = self.q_proj
            gv = ops.mhc_group_variant(qp.input_dim, qp.hidden_dim, x.shape[0], 3, x.dtype)
            if gv:
                plans = [m.plan() for m in (self.q_proj, self.k_proj, self.v_proj)]
                if all(p.fold for p in plans):
                    q, k, v = (t.view(n, L, -1) for t in ops.mhc_fused_group(x, plans, gv))
                    o = ops.attention(q, k, v, self.num_heads)
                    return self.out_proj.forward_tokens(o.view(n * L, -1))
        grp = ctx.plans.get(("group", id(self))) if (ctx is not None and opts.group_qkv) else None
        # a fused one-launch chain per projection beats sharing GEMM1 across q / k / v
        fused = opts.use_fused_mhc and ops.mhc_fused_supported(self.q_proj.input_dim, self.q_proj.hidden_dim, x.dtype)
        if grp is not None and not self.training and not fused:
            q, k, v = (t.view(n, L, -1) for t in self._qkv_grouped(x, grp))
            o = ops.attention(q, k, v, self.num_heads)
            return self.out_proj.forward_tokens(o.view(n * L, -1))
        if opts.parallel_qkv:
            main = torch.cuda.current_stream()
            if self._side is None:
                self._side = (torch.cuda.Stream(device=x.device), torch.cuda.Stream(device=x.device))
            sk, sv = self._side
            sk.wait_stream(main)
            sv.wait_stream(main)
            with torch.cuda.stream(sk):
                k = self.k_proj.forward_tokens(x)
            with torch.cuda.stream(sv):
                v = self.v_proj.forward_tokens(x)
            q = self.q_proj.forward_tokens(x)
            main.wait_stream(sk)
            main.wait_stream(sv)
            for t in (k, v):
                t.record_stream(main)
            x.record_stream(sk)
            x.record_stream(sv)
            q, k, v = q.view(n, L, -1), k.view(n, L, -1), v.view(n, L, -1)
        else:
            q = self.q_proj.forward_tokens(x).view(n, L, -1)
            k = self.k_proj.forward_tokens(x).view(n, L, -1)
            v = self.v_proj.forward_tokens(x).view(n, L, -1)
        o = ops.attention(q, k, v, self.num_heads)
        return self.out_proj.forward_tokens(o.view(n * L, -1))

    def _qkv_grouped(self, x: torch.Tensor, grp):
        """q / k / v mHC chains sharing x: ONE LayerNorm-statistics pass and ONE folded GEMM1
        with N = 3 * 2Hd (prep.PrepProgram lays the three sites' operands out contiguously);
        GEMM2 / GEMM3 / LN_post per site on column slices of the shared hidden activations."""
        mods, a1g, c1g, csg = grp
        ctx = current()
        ctx.join_prep()
        mean, rstd = ops.row_stats(x, 1e-5)
        h1 = ops.gemm(x, a1g, bias=c1g, act="gelu", a_mean=mean, a_rstd=rstd, b_colsum=csg)
        outs = []
        for j, m in enumerate(mods):
            p = ctx.plans[id(m)]
            w = 2 * p.Hd
            h2 = ops.gemm(h1[:, j * w:(j + 1) * w], p.w2, bias=p.bias2, act="gelu")
            yc = ops.gemm(x, p.wct, a2=h2, out_dtype=torch.float32)
            outs.append(ops.layernorm(yc, p.g_post, p.b_post, 1e-5, out_dtype=x.dtype))
        return outs

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False):
        """manifold_layers.py:386-434: (out [n, Lq, D], attn_weights [n, heads, Lq, Lk] or None).
        Self-attention without mask/weights runs the MFMA kernel; cross-attention, a key
        padding mask (True = ignore) or need_weights run hv_attention_general."""
        require_cuda(query, "MultiHeadManifoldAttention")
        general = key is not query or value is not query or key_padding_mask is not None or need_weights
        if self.training and not general:
            from . import train_model as TM
            n, L, D = query.shape
            x = query.reshape(n * L, D).to(resolve_dtype(self.q_proj)).contiguous()
            return TM.attention(self, x, n, TM.module_H(self)).view(n, L, D).to(query.dtype), None
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("hv_amd trains the self-attention call of TransformerEncoderBlock "
                                      "(vit_encoder_decoder.py:191); masked / cross / need_weights attention "
                                      "runs in eval mode or under torch.no_grad")
        n, Lq, D = query.shape
        dt = resolve_dtype(self.q_proj)
        with torch.no_grad():
            if not general:
                x = query.reshape(n * Lq, D).to(dt).contiguous()
                return self.forward_tokens(x, n).view(n, Lq, D).to(query.dtype), None
            Lk = key.shape[1]
            tok = lambda t: t.reshape(-1, D).to(dt).contiguous()   # noqa: E731
            q = self.q_proj.forward_tokens(tok(query)).view(n, Lq, D)
            k = self.k_proj.forward_tokens(tok(key)).view(n, Lk, D)
            v = self.v_proj.forward_tokens(tok(value)).view(n, Lk, D)
            o, w = ops.attention_general(q, k, v, self.num_heads, key_padding_mask, need_weights)
            out = self.out_proj.forward_tokens(o.view(n * Lq, D)).view(n, Lq, D).to(query.dtype)
        return out, w


class RMSNorm(nn.Module):
    """Reference manifold_layers.py:437-456."""

    def __init__(self, dim: int, eps: float = 1e-8):
        super().__init__()
        self.scale = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        require_cuda(x, "RMSNorm")
        if torch.is_grad_enabled() and (x.requires_grad or self.scale.requires_grad):
            from .train_fn import RMSNormFn
            shp = x.shape
            return RMSNormFn.apply(x.reshape(-1, shp[-1]), self.scale, self.eps).view(shp)
        return ops.rmsnorm(x.contiguous(), ops.f32(self.scale), self.eps)
