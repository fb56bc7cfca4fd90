"""Grouped per-forward parameter preparation (the "prep program" of a model).

The reference recomputes every parameter-only quantity on every forward: 76 Sinkhorn
projections and constrained matrices (manifold_layers.py:205-221), plus -- under GPU
autocast -- a cast of every weight and the eval-BN of every Conv-BN pair.  A PrepProgram
does all of it in a fixed, small number of launches over device tables:

    Sinkhorn group   2*iters+3 launches  (hv_sinkhorn_group_forward; histories written
                                          straight into each module's convergence_history)
    mHC prep group   4 launches          (hv_mhc_prep_group: Gc/u/Wc^T + fold GEMM + c1 + row sums)
    weight prep      1 launch            (hv_wprep_group: casts + Conv(+BN) reorder/fold)

and publishes the results into the forward's RunCtx.plans under the same keys the
per-module helpers use (id(mHC), ("conv", id(conv)), ("linear", id(linear))).  Output
buffers are persistent, so a captured hipGraph replays the whole program.

Conv/Linear layers are discovered on the first forward: a layer prepared outside the
program is registered and joins the grouped launch from the next forward on.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib as L
from . import tables
from .ops import SinkhornGroup, check, dtype_code, stream_ptr


def _param(t: torch.Tensor, what: str) -> torch.Tensor:
    t = t.detach()
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise TypeError(f"{what}: expected a contiguous fp32 parameter")
    return t


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


class PrepProgram:
    def __init__(self, mhc_mods: List[nn.Module], dtype: torch.dtype, device: torch.device, fold_max_d: int,
                 groups: Optional[Dict[int, Tuple]] = None):
        """groups: {key: (mHC, mHC, ...)} -- sites that read the same input (an attention's
        q/k/v projections): their folded GEMM1 operands (a1, c1, row sums) are laid out
        contiguously, so one GEMM with N = sum(2Hd) serves all of them (published in the plans
        under ("group", key))."""
        self.dtype, self.device = dtype, device
        self.mods = list(mhc_mods)
        self.fold_max_d = fold_max_d
        self.bf16 = dtype == torch.bfloat16
        lib = L.lib()
        hists = [m.sinkhorn.convergence_history for m in self.mods]
        for h, m in zip(hists, self.mods):
            if not (h.is_cuda and h.dtype == torch.float32 and h.is_contiguous()
                    and h.numel() >= m.sinkhorn.num_iterations):
                raise TypeError("convergence_history must be a contiguous fp32 device buffer")
        self.sk = SinkhornGroup([_param(m.H_res_raw, "H_res_raw") for m in self.mods],
                                [m.sinkhorn.num_iterations for m in self.mods], device,
                                self.mods[0].sinkhorn.epsilon, self.mods[0].sinkhorn.tau, hists=hists)
        # ---- mHC prep entries + persistent outputs
        n = len(self.mods)
        self.mentries = (L.MhcPrepEntry * n)()
        offs, total = [], 0
        for m in self.mods:
            offs.append(total)
            total += (lib.hv_mhc_prep_scratch_floats(m.input_dim, m.hidden_dim) + 63) // 64 * 64
        self.scratch = torch.empty(max(total, 1), device=device, dtype=torch.float32)
        self.mout: List[Tuple] = []
        tot = [0, 0, 0, 0]
        blk = (L.i32 * 4)()
        self.wcasts: List[Tuple[torch.Tensor, torch.Tensor]] = []     # (src, dst) for the weight group
        # contiguous GEMM1 operands for grouped sites
        self.groups: Dict[object, Tuple] = {}
        slot: Dict[int, Tuple] = {}
        present = {id(m) for m in self.mods}
        for gk, members in (groups or {}).items():
            ms = list(members)
            D0, H0 = ms[0].input_dim, ms[0].hidden_dim
            if not all(id(m) in present and m.input_dim == D0 and m.hidden_dim == H0 for m in ms):
                continue
            if not (D0 <= fold_max_d and H0 % 32 == 0):
                continue
            g = len(ms)
            a1g = torch.empty((g * 2 * H0, D0), device=device, dtype=dtype)
            c1g = torch.empty(g * 2 * H0, device=device, dtype=torch.float32)
            csg = torch.empty(g * 2 * H0, device=device, dtype=torch.float32)
            for j, m in enumerate(ms):
                sl = slice(j * 2 * H0, (j + 1) * 2 * H0)
                slot[id(m)] = (a1g[sl], c1g[sl], csg[sl])
            self.groups[gk] = (tuple(ms), a1g, c1g, csg)
        for i, m in enumerate(self.mods):
            D, Hd = m.input_dim, m.hidden_dim
            fold = D <= fold_max_d and Hd % 32 == 0
            if id(m) in slot:
                a1, c1, cs = slot[id(m)]
            else:
                a1 = torch.empty((2 * Hd, D) if fold else (Hd, D), device=device, dtype=dtype)
                c1 = torch.empty(2 * Hd if fold else Hd, device=device, dtype=torch.float32)
                cs = torch.empty(a1.shape[0], device=device, dtype=torch.float32)
            wct = torch.empty((D, D + Hd), device=device, dtype=dtype)
            w1 = _param(m.mlp[0].weight, "mlp[0].weight")
            w2 = _param(m.mlp[3].weight, "mlp[3].weight")
            w2c = self._cast_target(w2)
            w1c = None if fold else self._cast_target(w1)
            e = self.mentries[i]
            e.h_pre_raw = _param(m.H_pre_raw, "H_pre_raw").data_ptr()
            e.h_post_raw = _param(m.H_post_raw, "H_post_raw").data_ptr()
            e.h_res = self.sk.outs[i].data_ptr()
            e.gamma_pre = _param(m.norm_pre.weight, "norm_pre.weight").data_ptr()
            e.beta_pre = _param(m.norm_pre.bias, "norm_pre.bias").data_ptr()
            e.w1 = w1.data_ptr()
            e.b1 = _param(m.mlp[0].bias, "mlp[0].bias").data_ptr()
            e.a1, e.c1, e.wct = a1.data_ptr(), c1.data_ptr(), wct.data_ptr()
            e.scratch = self.scratch.data_ptr() + 4 * offs[i]
            e.cs = cs.data_ptr()
            e.D, e.Hd, e.fold = D, Hd, int(fold)
            lib.hv_mhc_prep_blocks(D, Hd, int(fold), blk)
            for p in range(4):
                e.blk[p] = tot[p]
                tot[p] += blk[p]
            self.mout.append((fold, a1, c1, wct, w1c, w2c, cs))
        self.mtotals = (L.i32 * 4)(*tot)
        self.mtable = tables.upload(self.mentries, device, self, "mhc_prep")
        # ---- weight prep (casts of the mHC MLP weights + registered convs / linears)
        self.convs: Dict[int, Tuple] = {}
        self.linears: Dict[int, Tuple] = {}
        self.wtable = None
        self._wdirty = True
        self._sides: Dict[int, torch.cuda.Stream] = {}   # run(overlap=True): per forward stream
        self.param_ptrs = self._ptr_key()

    # ------------------------------------------------------------------ registration
    def _cast_target(self, w: torch.Tensor) -> torch.Tensor:
        if not self.bf16:
            return w                                  # fp32 mode: use the parameter itself
        out = torch.empty(w.shape, device=self.device, dtype=self.dtype)
        self.wcasts.append((w, out))
        self._wdirty = True
        return out

    def add_conv(self, conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d]):
        cout, cin, k, _ = conv.weight.shape
        kk = k * k * cin
        epc = 8 if self.bf16 else 4
        ldk = (kk + epc - 1) // epc * epc
        w = torch.empty((cout, ldk), device=self.device, dtype=self.dtype)
        scale = bias_out = None
        if bn is not None:
            scale = torch.empty(cout, device=self.device, dtype=torch.float32)
            bias_out = torch.empty(cout, device=self.device, dtype=torch.float32)
        bias = bias_out if bn is not None else (None if conv.bias is None else _param(conv.bias, "conv.bias"))
        self.convs[id(conv)] = (conv, bn, w, scale, bias_out, (w[:, :kk], scale, bias))
        self._wdirty = True
        return self.convs[id(conv)][5]

    def add_linear(self, lin: nn.Linear):
        wt = _param(lin.weight, "linear.weight")
        w = self._cast_target(wt)
        val = (w, None if lin.bias is None else _param(lin.bias, "linear.bias"))
        self.linears[id(lin)] = (lin, val)
        return val

    def _build_wtable(self):
        ents = []
        for src, dst in self.wcasts:
            ents.append(("cast", src, dst))
        for conv, bn, w, scale, bias_out, _ in self.convs.values():
            ents.append(("conv", conv, bn, w, scale, bias_out))
        if not ents:
            self.wtable = None
            self._wdirty = False
            return
        lib = L.lib()
        tab = (L.WprepEntry * len(ents))()
        tot = 0
        for i, ent in enumerate(ents):
            e = tab[i]
            if ent[0] == "cast":
                _, src, dst = ent
                e.src, e.dst, e.n, e.kind = src.data_ptr(), dst.data_ptr(), src.numel(), 0
                e.dtype = dtype_code(dst.dtype)
                nb = lib.hv_wprep_blocks(0, src.numel(), 0, 0)
            else:
                _, conv, bn, w, scale, bias_out = ent
                cout, cin, k, _ = conv.weight.shape
                e.src = _param(conv.weight, "conv.weight").data_ptr()
                e.dst, e.n, e.kind, e.dtype = w.data_ptr(), cout, 1, dtype_code(w.dtype)
                e.cin, e.k, e.ldk = cin, k, w.shape[1]
                if bn is not None:
                    e.gamma = _param(bn.weight, "bn.weight").data_ptr()
                    e.beta = _param(bn.bias, "bn.bias").data_ptr()
                    e.mean = _param(bn.running_mean, "bn.running_mean").data_ptr()
                    e.var = _param(bn.running_var, "bn.running_var").data_ptr()
                    e.eps = bn.eps
                    e.cbias = _ptr(None if conv.bias is None else _param(conv.bias, "conv.bias"))
                    e.scale_out, e.bias_out = scale.data_ptr(), bias_out.data_ptr()
                nb = lib.hv_wprep_blocks(1, cout, cin, k)
            e.blk = tot
            tot += nb
        self.wentries = tab
        self.wtotal = tot
        self.wtable = tables.upload(tab, self.device, self, "wprep")
        self._wdirty = False

    # ------------------------------------------------------------------ run
    def _run_mhc(self, lib) -> None:
        self.sk.run()
        check(lib.hv_mhc_prep_group(self.mtable.data_ptr(), len(self.mods), dtype_code(self.dtype),
                                    self.mtotals, stream_ptr()), "hv_mhc_prep_group")

    def _ptr_key(self):
        return tuple(p.data_ptr() for m in self.mods for p in m.parameters(recurse=True))

    def valid_for(self, mods, dtype) -> bool:
        return dtype == self.dtype and len(mods) == len(self.mods) and all(
            a is b for a, b in zip(mods, self.mods)) and self._ptr_key() == self.param_ptrs

    def run(self, ctx, overlap: bool = False) -> None:
        """Recompute everything parameter-only and publish the plans into ctx.

        overlap: run the Sinkhorn group and the mHC prep (latency-bound, ~1.6 ms at base 640)
        on a side stream forked from the current one, beside the weight prep (HBM-bound) and the
        layers before the first mHC site; ctx.join_prep() -- called by the first mHC plan lookup
        and at the end of the forward -- joins it back (a captured graph gets the fork/join as
        two branches)."""
        from .manifold import MhcPlan
        lib = L.lib()
        if overlap:
            main = torch.cuda.current_stream()
            # one side stream per forward stream (as runtime.Branches): a forward on another
            # stream -- another thread's eager forward beside a graph capture -- never shares it
            side = self._sides.get(main.cuda_stream)
            if side is None:
                side = self._sides.setdefault(main.cuda_stream, torch.cuda.Stream(device=self.device))
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self._run_mhc(lib)
                ev = torch.cuda.Event()
                ev.record(side)
            ctx.prep_event = ev
        else:
            self._run_mhc(lib)
        if self._wdirty:
            self._build_wtable()
        if self.wtable is not None:
            check(lib.hv_wprep_group(self.wtable.data_ptr(), len(self.wentries), self.wtotal, stream_ptr()),
                  "hv_wprep_group")
        for m, (fold, a1, c1, wct, w1c, w2c, cs) in zip(self.mods, self.mout):
            ctx.plans[id(m)] = MhcPlan(
                D=m.input_dim, Hd=m.hidden_dim, fold=fold, dtype=self.dtype, b1=a1, c1=c1,
                w1=w1c, bias1=None if fold else m.mlp[0].bias.detach(), w2=w2c, bias2=m.mlp[3].bias.detach(),
                wct=wct, g_post=m.norm_post.weight.detach(), b_post=m.norm_post.bias.detach(), cs=cs)
        for gk, grp in self.groups.items():
            ctx.plans[("group", gk)] = grp
        for conv, bn, w, scale, bias_out, val in self.convs.values():
            ctx.plans[("conv", id(conv))] = val
        for lin, val in self.linears.values():
            ctx.plans[("linear", id(lin))] = val
