"""Grouped per-forward coefficient preparation of the TRAINING step.

The training forward of every mHC site needs the folded operands of manifold_layers.py:223-280
(Gc, u, Wc^T, A1 = Gc W1^T, c1 = W1 u + b1, the compute-dtype W2) and its backward a few
transposed copies of parameter-sized matrices (A1, Wc, W2^T, Gc^T, W1^T).  Built per site they
were ~15 launches per site -- about 1,100 launches of a few microseconds each per step at base
640 (k_cast, k_transpose_cast, k_gemv, the per-site prep).  A TrainPrep computes all of them for
all 76 sites in 5 launches per forward: the inference prep group (hv_mhc_prep_group: column sums,
Gc / u / Wc^T, the fold GEMM + c1, row sums) over the training Sinkhorn outputs, then ONE
hv_transpose_group launch for every transposed / cast copy.  Outputs are persistent buffers
(stable pointers for a captured training graph); one forward's coefficients are consumed by its
backward, which checks a generation counter (a second forward before the first backward would
overwrite them, and raises instead of differentiating the wrong values).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List

import torch

from . import _lib as L
from . import tables
from .ops import check, dtype_code, stream_ptr


@dataclass
class TrainCoef:
    a1t: torch.Tensor    # [2Hd, D] dt   GEMM1 operand (A1^T)
    c1: torch.Tensor     # [2Hd] fp32    GEMM1 bias W1 u + b1
    w2: torch.Tensor     # [Hd, 2Hd] dt  GEMM2 operand
    wct: torch.Tensor    # [D, D+Hd] dt  GEMM3 operand (centred [H_res ; H_post]^T)
    a1: torch.Tensor     # [D, 2Hd] dt   backward dz = dpre1 A1
    wc: torch.Tensor     # [D+Hd, D] dt  backward dyc -> d[x | h2]
    w2t: torch.Tensor    # [2Hd, Hd] dt  backward dpre2 -> dh1
    gct: torch.Tensor    # [Hd, D] pdt   backward dW1 = dA1t Gc
    w1t: torch.Tensor    # [Hd, 2Hd] fp32 backward du = W1^T dc1
    gc: torch.Tensor     # [D, Hd] fp32
    u: torch.Tensor      # [Hd] fp32
    owner: "TrainPrep"
    gen: int = 0


class TrainPrep:
    def __init__(self, mods: List[torch.nn.Module], h_res: List[torch.Tensor], dtype: torch.dtype):
        lib = L.lib()
        self.mods, self.dtype = list(mods), dtype
        dev = h_res[0].device
        pdt = torch.bfloat16 if dtype == torch.bfloat16 else torch.float32
        self.h_ptrs = tuple(h.data_ptr() for h in h_res)
        self.h_res = list(h_res)               # the Sinkhorn outputs the prep table reads
        self.param_ptrs = self._param_key()
        n = len(self.mods)
        offs, total = [], 0
        for m in self.mods:
            offs.append(total)
            total += (lib.hv_mhc_prep_scratch_floats(m.input_dim, m.hidden_dim) + 63) // 64 * 64
        self.scratch = torch.empty(max(total, 1), device=dev, dtype=torch.float32)
        self.mentries = (L.MhcPrepEntry * n)()
        tot = [0, 0, 0, 0]
        blk = (L.i32 * 4)()
        self.coefs: Dict[int, TrainCoef] = {}
        self._keep: List[torch.Tensor] = []    # every buffer a device table points at stays referenced
        trans = []
        emp = lambda *shape, dt=dtype: torch.empty(shape, device=dev, dtype=dt)   # noqa: E731
        for i, (m, h) in enumerate(zip(self.mods, h_res)):
            D, Hd = m.input_dim, m.hidden_dim
            if Hd % 32 or h.dtype != torch.float32 or not h.is_contiguous():
                raise ValueError("TrainPrep: every site folds (Hd % 32 == 0), H_res contiguous fp32")
            W1, W2 = m.mlp[0].weight.detach(), m.mlp[3].weight.detach()
            a1t, c1, cs, wct = emp(2 * Hd, D), emp(2 * Hd, dt=torch.float32), emp(2 * Hd, dt=torch.float32), emp(D, D + Hd)
            sc = self.scratch[offs[i]:]
            gc, u = sc[:D * Hd].view(D, Hd), sc[D * Hd:D * Hd + Hd]
            co = TrainCoef(a1t=a1t, c1=c1, w2=emp(Hd, 2 * Hd) if dtype != torch.float32 else W2, wct=wct,
                           a1=emp(D, 2 * Hd), wc=emp(D + Hd, D), w2t=emp(2 * Hd, Hd), gct=emp(Hd, D, dt=pdt),
                           w1t=emp(Hd, 2 * Hd, dt=torch.float32), gc=gc, u=u, owner=self)
            self.coefs[id(m)] = co
            self._keep.append(cs)              # written by the prep's row-sum phase: must outlive the table
            e = self.mentries[i]
            e.h_pre_raw, e.h_post_raw = m.H_pre_raw.data_ptr(), m.H_post_raw.data_ptr()
            e.h_res = h.data_ptr()
            e.gamma_pre, e.beta_pre = m.norm_pre.weight.data_ptr(), m.norm_pre.bias.data_ptr()
            e.w1, e.b1 = W1.data_ptr(), m.mlp[0].bias.data_ptr()
            e.a1, e.c1, e.wct, e.cs = a1t.data_ptr(), c1.data_ptr(), wct.data_ptr(), cs.data_ptr()
            e.scratch = sc.data_ptr()
            e.D, e.Hd, e.fold = D, Hd, 1
            lib.hv_mhc_prep_blocks(D, Hd, 1, blk)
            for p in range(4):
                e.blk[p] = tot[p]
                tot[p] += blk[p]
            trans += [(a1t, co.a1, 1), (wct, co.wc, 1), (W2, co.w2t, 1), (gc, co.gct, 1), (W1, co.w1t, 1)]
            if dtype != torch.float32:
                trans.append((W2, co.w2, 0))
        self.mtotals = (L.i32 * 4)(*tot)
        self.mtable = tables.upload(self.mentries, dev, self, "mhc_prep")
        self.tentries = (L.TransposeEntry * len(trans))()
        tb = 0
        for j, (x, y, tr) in enumerate(trans):
            t = self.tentries[j]
            rows, cols = x.shape
            t.x, t.y, t.rows, t.cols = x.data_ptr(), y.data_ptr(), rows, cols
            t.x_dtype, t.y_dtype, t.transpose, t.blk = dtype_code(x.dtype), dtype_code(y.dtype), tr, tb
            tb += lib.hv_transpose_blocks(rows, cols)
        self.ttotal = tb
        self.ttable = tables.upload(self.tentries, dev, self, "transpose")
        self.gen = 0

    def _param_key(self):
        return tuple(p.data_ptr() for m in self.mods for p in m.parameters(recurse=True))

    def valid_for(self, mods, h_res, dtype) -> bool:
        return (dtype == self.dtype and len(mods) == len(self.mods) and all(a is b for a, b in zip(mods, self.mods))
                and tuple(h.data_ptr() for h in h_res) == self.h_ptrs and self._param_key() == self.param_ptrs)

    def run(self) -> Dict[int, TrainCoef]:
        """Recompute every site's coefficients from the current parameters and H_res buffers."""
        lib = L.lib()
        check(lib.hv_mhc_prep_group(self.mtable.data_ptr(), len(self.mods), dtype_code(self.dtype), self.mtotals,
                                    stream_ptr()), "hv_mhc_prep_group")
        check(lib.hv_transpose_group(self.ttable.data_ptr(), len(self.tentries), self.ttotal, stream_ptr()),
              "hv_transpose_group")
        self.gen += 1
        for c in self.coefs.values():
            c.gen = self.gen
        return self.coefs
