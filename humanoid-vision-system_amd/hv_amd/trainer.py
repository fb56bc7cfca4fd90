"""Training step driver: forward in training mode with YOLOLoss,
backward, data-parallel gradient all-reduce over RCCL overlapped with the backward, per-group
gradient clipping and AdamW -- the last two as HIP kernels over a device parameter table.

Reference semantics followed:
  * loss: YOLOLoss total_loss (yolo_head.py:374-465) from HybridVisionSystem.forward(...,
    compute_loss=True) (hybrid_vision.py:222-367);
  * clipping: mhc_trainer.py:342-383 -- torch.nn.utils.clip_grad_norm_ semantics, group
    'mhc' (name contains 'mhc' or 'H_') at mhc_max_norm=0.5, the rest at max_grad_norm=1.0;
  * optimizer: optimizer.py:131-191 -- AdamW (decoupled decay before the Adam update),
    lr 1e-3, weight_decay 1e-4, betas (0.9, 0.999), eps 1e-8 (the 'manifold' branch is empty
    because _get_param_name returns str(shape));
  * DDP as intended by scripts/train.py: gradients averaged over ranks, rank-0 buffers (BN
    running stats, mHC monitors) broadcast before every forward (broadcast_buffers=True),
    per-replica BN statistics (no SyncBatchNorm).

Gradients live in ONE flat fp32 buffer (each param.grad is a view), bucketed in reverse
registration order (the order the backward produces them); a bucket's all-reduce is launched
from the post-accumulate hook of its last parameter, so RCCL traffic over xGMI overlaps the
rest of the backward.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, List, Optional, Sequence

import torch
from torch.autograd.graph import increment_version
import torch.distributed as dist

from . import _lib as L
from ._lib import check, stream_ptr

Tensor = torch.Tensor


def mhc_group(name: str) -> int:
    """Clipping group of a parameter (mhc_trainer.py:356-360): 0 = mHC, 1 = other."""
    return 0 if ("mhc" in name.lower() or "H_" in name) else 1


class GradBuckets:
    """Flat gradient storage + bucketed, hook-driven all-reduce (average over ranks).

    During the backward every parameter's .grad starts as None, so autograd STORES the
    gradient its producer computed (no accumulate kernel per parameter, which at 1,149
    parameters was ~1,250 tiny `add` launches per step).  When a bucket's last parameter has
    its gradient, one segmented-copy launch (hv_copy_segments) moves the bucket into its span of
    the flat buffer and, with world > 1, that span's all-reduce starts (RCCL over xGMI) while the
    rest of the backward runs.  finish() leaves every param.grad as a view of the flat buffer
    (zero for parameters that got no gradient) for the clipping / AdamW table.

    Works on any device / process-group backend: the CPU `gloo` tests drive it with plain
    torch modules, the GPU trainer with RCCL ('nccl')."""

    def __init__(self, named_params: Sequence, bucket_bytes: int = 64 << 20, group=None):
        self.params = [p for _, p in named_params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        self.offsets: Dict[int, int] = {}
        self.views: List[Tensor] = []
        off = 0
        for p in self.params:
            self.offsets[id(p)] = off
            v = self.flat[off:off + p.numel()].view_as(p)
            self.views.append(v)
            p.grad = v
            off += p.numel()
        # buckets over the reverse order (backward produces the last layers first)
        self.buckets: List[List[Tensor]] = []
        cur, cur_bytes = [], 0
        for p in reversed(self.params):
            cur.append(p)
            cur_bytes += p.numel() * 4
            if cur_bytes >= bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self._pending: List = []
        self._ready = [set() for _ in self.buckets]
        self._flushed = [False] * len(self.buckets)
        self._reduced = [False] * len(self.buckets)
        # Collective order must be identical on every rank.  A bucket is reduced from the hooks
        # (overlapping the backward) only if EVERY rank completed it through the hooks on the
        # previous step (`agreed`, all-reduced MIN in finish()), and agreed buckets are issued in
        # bucket order; finish() then issues the agreed buckets still open, then the others, each
        # in bucket order.  Step 1 (nothing agreed yet) reduces everything in finish().
        self.agreed = [False] * len(self.buckets)
        self._next = 0
        # the gradients were pre-divided by world (HVTrainer scales the loss by 1/world, exact for
        # power-of-two worlds): the all-reduce then sums, with no per-bucket division pass
        self.prescaled = False
        # device-side 'received a gradient' flags (OR over ranks), read by the clipping / AdamW
        # kernels -- no host round trip; the host copy (`received`) is materialised on demand
        self.active_dev: Optional[Tensor] = None
        self._flags_key = None
        self._flags_local: Optional[Tensor] = None
        self._flag_reads: List = []            # (event, pinned host copy) of reduced flags, oldest first
        self._received_host: Optional[List[bool]] = None
        # which parameters received a gradient this step: the optimizer skips the others like
        # torch.optim skips grad=None (optimizer.py:144)
        self._received_local = [False] * len(self.params)
        self._index = {id(p): i for i, p in enumerate(self.params)}
        # the engine runs a leaf's hooks even when its producer returned None for it (e.g. the
        # grouped Sinkhorn's unused final-fusion projection), so receipt is read from the
        # gradient itself in a tensor hook; bucket readiness is counted in the post-accumulate hook
        self._hooks = [p.register_hook(self._flag_hook(i)) for i, p in enumerate(self.params)]
        self._hooks += [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        # zero-copy gradients: the largest producers (weight-gradient GEMMs, ops_train.grad_out)
        # write their first contribution of a step straight into the parameter's flat view, which
        # autograd then stores as .grad -- the bucket flush skips it (no hv_copy_segments bytes)
        self._claimed = [False] * len(self.params)
        for i, p in enumerate(self.params):
            p._hv_grad_claim = self._claimer(i)

    def _claimer(self, idx: int):
        off, p = self.offsets[id(self.params[idx])], self.params[idx]
        n, shape = p.numel(), tuple(p.shape)

        def claim():
            if self._claimed[idx]:
                return None
            self._claimed[idx] = True
            return self.flat[off:off + n].view(shape)       # a fresh view object (autograd may steal it)
        return claim

    def _flag_hook(self, idx: int):
        def hook(g):
            if g is not None:
                self._received_local[idx] = True
        return hook

    def _span(self, i: int):
        b = self.buckets[i]
        lo = min(self.offsets[id(p)] for p in b)
        hi = max(self.offsets[id(p)] + p.numel() for p in b)
        return lo, hi

    def _flush(self, params) -> None:
        """Move the stored (non-view) gradients of `params` into the flat buffer."""
        pairs = []
        for p in params:
            g = p.grad
            v = self.views[self._index[id(p)]]
            if g is None or g.data_ptr() == v.data_ptr():
                continue
            if g.dtype != torch.float32 or not g.is_contiguous():
                g = g.float().contiguous()
            pairs.append((g, v))
        if not pairs:
            return
        if pairs[0][1].is_cuda:
            from . import _lib as L
            segs = (L.CopySegment * len(pairs))()
            for j, (g, v) in enumerate(pairs):
                segs[j].src, segs[j].dst, segs[j].bytes = g.data_ptr(), v.data_ptr(), g.numel() * 4
            check(L.lib().hv_copy_segments(segs, len(pairs), stream_ptr()), "hv_copy_segments")
        else:                                   # CPU (gloo tests): host copies
            with torch.no_grad():
                for g, v in pairs:
                    v.copy_(g)
        for g, v in pairs:                       # keep the sources alive until the copy ran
            if g.is_cuda:
                g.record_stream(torch.cuda.current_stream())

    def _reduce(self, i: int) -> None:
        self._reduced[i] = True
        if self.world > 1:
            lo, hi = self._span(i)
            view = self.flat[lo:hi]
            if not self.prescaled:
                view.div_(self.world)
            self._pending.append(dist.all_reduce(view, group=self.group, async_op=True))

    def _issue_agreed(self) -> None:
        """Reduce the agreed buckets in bucket order, as far as they are flushed."""
        while self._next < len(self.buckets):
            i = self._next
            if self.agreed[i]:
                if not self._flushed[i]:
                    return
                self._reduce(i)
            self._next += 1

    def _on_grad(self, p: Tensor):
        i = self.bucket_of[id(p)]
        self._ready[i].add(id(p))
        if len(self._ready[i]) == len(self.buckets[i]) and not self._flushed[i]:
            self._flush(self.buckets[i])
            self._flushed[i] = True
            for q in self.buckets[i]:            # free the stored gradients now
                q.grad = self.views[self._index[id(q)]]
            self._issue_agreed()

    def zero(self):
        """Start a step: flat buffer zeroed (one fill), every param.grad set to None so the
        backward stores rather than accumulates."""
        self.flat.zero_()
        for p in self.params:
            p.grad = None
        self._claimed = [False] * len(self.params)
        self._received_local = [False] * len(self.params)
        self._received_host = None
        self._ready = [set() for _ in self.buckets]
        self._flushed = [False] * len(self.buckets)
        self._reduced = [False] * len(self.buckets)
        self._next = 0
        self._pending = []
        self._consume_flag_reads(lag=2)

    @property
    def received(self) -> List[bool]:
        """Per-parameter 'received a gradient this step' (OR over ranks), on the host.  The step
        itself only uses the device copy (`active_dev`); reading this synchronises with it."""
        if self._received_host is None:
            if self.active_dev is None:
                return list(self._received_local)
            self._received_host = [bool(v) for v in self.active_dev.tolist()]
        return self._received_host

    def _consume_flag_reads(self, lag: int) -> None:
        """Apply the reduced 'bucket completed through the hooks' flags of the step `lag` steps
        back as the agreed set.  Every rank applies the same step's flags at the same point, so
        the collective order stays identical; lag 2 means the event has long completed (the host
        never waits on the current step's GPU work)."""
        while len(self._flag_reads) >= lag:
            ev, host = self._flag_reads.pop(0)
            if ev is not None:
                ev.synchronize()
            n = len(self.params)
            self.agreed = [v == 0 for v in host[n:].tolist()]

    def finish(self):
        """Flush and reduce the buckets not reduced from the hooks -- the agreed ones still open
        first, then the rest, each in bucket order, so every rank issues the same collectives in
        the same order -- wait for the all-reduces, and point every param.grad at its flat view.
        With world > 1 the received-gradient flags are OR-ed over ranks (one small all-reduce),
        so every replica skips exactly the parameters no rank produced a gradient for, and the
        buckets every rank completed through the hooks become next step's agreed set."""
        hooked = [self._flushed[i] for i in range(len(self.buckets))]
        for agreed_pass in (True, False):
            for i, b in enumerate(self.buckets):
                if self.agreed[i] != agreed_pass or self._reduced[i]:
                    continue
                if not self._flushed[i]:
                    self._flush(b)
                    self._flushed[i] = True
                self._reduce(i)
        for w in self._pending:
            w.wait()
        self._pending = []
        for p, v in zip(self.params, self.views):
            p.grad = v
        n = len(self.params)
        key = tuple(self._received_local) + tuple(hooked)
        if key != self._flags_key:              # new local flags: one async upload (then cached)
            from .ops import upload_bytes
            host = torch.tensor([int(r) for r in self._received_local] + [1 - int(h) for h in hooked],
                                dtype=torch.int32)
            self._flags_local = upload_bytes(host.numpy().tobytes(), self.flat.device, torch.int32)
            self._flags_key = key
        if self.world > 1:
            flags = self._flags_local.clone()
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=self.group)
            self.active_dev = flags[:n]
            if flags.is_cuda:                   # read back two steps later, without a stall
                host = torch.empty(flags.shape, dtype=flags.dtype).pin_memory()
                host.copy_(flags, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._flag_reads.append((ev, host))
            else:                               # gloo on CPU: the reduce is done, apply it now
                self._flag_reads.append((None, flags.clone()))
                self._consume_flag_reads(lag=1)
        else:
            self.active_dev = self._flags_local[:n]
            self.agreed = hooked


class FusedAdamW:
    """Per-group grad-norm clipping + AdamW as HIP kernels over a device table (hv_grad_norms,
    hv_adamw); no host synchronisation.  Which parameters take part in a step ('received a
    gradient', torch.optim's grad-is-None skip) is a DEVICE flag array read by the kernels, so a
    data-parallel step never waits on the host for it and the whole step is graph-capturable."""

    def __init__(self, named_params: Sequence, lr: float = 1e-3, weight_decay: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, max_norms=(0.5, 1.0)):
        self.named = [(n, p) for n, p in named_params if p.requires_grad]
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.max_norms = list(max_norms)
        dev = self.named[0][1].device
        self.exp_avg = [torch.zeros_like(p) for _, p in self.named]
        self.exp_avg_sq = [torch.zeros_like(p) for _, p in self.named]
        self.step_count = 0
        # per-parameter step counts (reference / torch.optim state['step']) live on the device,
        # advanced by the active flags; param_steps reads them back on demand
        self._steps_dev = torch.zeros(len(self.named), device=self.named[0][1].device, dtype=torch.int32)
        self._active_cache = (None, None)
        self.norms = torch.zeros(len(self.max_norms), device=dev, dtype=torch.float32)
        self.coefs = torch.ones(len(self.max_norms), device=dev, dtype=torch.float32)
        self._table = None
        self._key = None
        self.device = dev
        # lr, beta1, beta2, eps, weight_decay as a DEVICE array read by hv_adamw_dev: a scheduler
        # changing lr every step (mhc_trainer.py:275) updates it by a small async copy, so a
        # captured training graph keeps replaying instead of re-capturing per value
        self._hyper = torch.zeros(5, device=dev, dtype=torch.float32)
        self._hyper_vals = None
        self._hyper_ring = []               # (pinned host [5], event) staging slots
        self._hyper_slot = 0

    def hyper_values(self):
        return (float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps), float(self.wd))

    def sync_hyper(self) -> None:
        """Upload the hyper-parameters when they changed since the last upload, asynchronously on
        the current stream (never inside a graph capture: the replay reads the device array)."""
        vals = self.hyper_values()
        if vals == self._hyper_vals:
            return
        if self._hyper.device.type != "cuda":
            self._hyper.copy_(torch.tensor(vals, dtype=torch.float32))
        else:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedAdamW.sync_hyper inside a graph capture")
            if not self._hyper_ring:
                self._hyper_ring = [(torch.empty(5, dtype=torch.float32).pin_memory(), None) for _ in range(4)]
            pin, ev = self._hyper_ring[self._hyper_slot]
            if ev is not None:
                ev.synchronize()            # that slot's previous copy has left the staging buffer
            pin.copy_(torch.tensor(vals, dtype=torch.float32))
            self._hyper.copy_(pin, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._hyper_ring[self._hyper_slot] = (pin, ev)
            self._hyper_slot = (self._hyper_slot + 1) % len(self._hyper_ring)
        self._hyper_vals = vals

    @property
    def param_steps(self) -> List[int]:
        return [int(v) for v in self._steps_dev.tolist()]

    @param_steps.setter
    def param_steps(self, steps: Sequence[int]) -> None:
        self._steps_dev.copy_(torch.tensor([int(v) for v in steps], dtype=torch.int32))

    def _build(self):
        lib = L.lib()
        ents = (L.ParamEntry * len(self.named))()
        blk = 0
        for i, (name, p) in enumerate(self.named):
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise TypeError(f"{name}: FusedAdamW needs contiguous fp32 parameters")
            e = ents[i]
            e.param = p.data_ptr()
            e.grad = p.grad.data_ptr() if p.grad is not None else None
            e.exp_avg, e.exp_avg_sq = self.exp_avg[i].data_ptr(), self.exp_avg_sq[i].data_ptr()
            e.n = p.numel()
            e.group = mhc_group(name)
            e.blk = blk
            blk += lib.hv_param_blocks(p.numel())
        self._blocks = blk
        from . import tables
        self._table = tables.upload(ents, self.device, self, "params")
        self._work = torch.empty(2 * blk, device=self.device, dtype=torch.float32)

    def _active_tensor(self, active) -> Tensor:
        """Device int32 [count] flags from a device tensor (used as is), a host sequence (uploaded
        once per distinct value) or None (every parameter with a gradient)."""
        if isinstance(active, torch.Tensor):
            if active.numel() != len(self.named) or active.dtype != torch.int32 or not active.is_cuda:
                raise ValueError("active: device int32 tensor with one flag per parameter")
            return active
        key = tuple(bool(a) for a in active) if active is not None else (True,) * len(self.named)
        if self._active_cache[0] != key:
            from .ops import upload_bytes
            host = torch.tensor([int(a) for a in key], dtype=torch.int32)
            self._active_cache = (key, upload_bytes(host.numpy().tobytes(), self.device, torch.int32))
        return self._active_cache[1]

    def step(self, clip: bool = True, active=None):
        """active[i] false = parameter i got no gradient this step: no clipping contribution,
        no weight decay, no moment update (torch.optim's grad-is-None skip)."""
        key = tuple((p.data_ptr(), None if p.grad is None else p.grad.data_ptr()) for _, p in self.named)
        if key != self._key:
            self._build()
            self._key = key
        act = self._active_tensor(active)
        lib = L.lib()
        self.step_count += 1
        self._steps_dev.add_(act)
        coefs = None
        if clip:
            mx = (C.c_float * len(self.max_norms))(*self.max_norms)
            check(lib.hv_grad_norms(self._table.data_ptr(), len(self.named), self._blocks, len(self.max_norms), mx,
                                    self.norms.data_ptr(), self.coefs.data_ptr(), self._work.data_ptr(),
                                    act.data_ptr(), stream_ptr()), "hv_grad_norms")
            coefs = self.coefs.data_ptr()
        if not (self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            self.sync_hyper()
        check(lib.hv_adamw_dev(self._table.data_ptr(), len(self.named), self._blocks, coefs, self._hyper.data_ptr(),
                               self._steps_dev.data_ptr(), act.data_ptr(), stream_ptr()), "hv_adamw_dev")
        # the kernel wrote the parameters behind autograd's back: bump their version counters as
        # an in-place torch update would, so frozen coefficients / captured graphs (VersionWatch)
        # see the new weights (every parameter: the skipped ones are unchanged but a version
        # bump is harmless, and knowing which were skipped would need the device flags)
        self.bump_versions()

    def bump_versions(self) -> None:
        increment_version([p for _, p in self.named])

    # ---- torch.optim-compatible state (checkpoints load into / from torch.optim.AdamW)
    def state_dict(self) -> Dict:
        """torch.optim layout; loads into torch.optim.AdamW and into the reference
        ManifoldAwareOptimizer (optimizer.py:31-70: its param group also carries mhc_params and
        manifold_update_freq, read by step() at :125).  Parameters that never received a
        gradient have no state, as in torch."""
        steps = self.param_steps
        state = {i: {"step": torch.tensor(float(steps[i])), "exp_avg": self.exp_avg[i],
                     "exp_avg_sq": self.exp_avg_sq[i]} for i in range(len(self.named)) if steps[i] > 0}
        return {"state": state,
                "param_groups": [{"lr": self.lr, "betas": tuple(self.betas), "eps": self.eps,
                                  "weight_decay": self.wd, "amsgrad": False, "maximize": False,
                                  "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                                  "mhc_params": {"mhc_lr_scale": 0.5, "project_iterations": 20,
                                                 "strict_double_stochastic": True},
                                  "manifold_update_freq": 100,
                                  "params": list(range(len(self.named)))}]}

    def load_state_dict(self, sd: Dict) -> None:
        g = sd["param_groups"][0]
        self.lr, self.betas, self.eps, self.wd = g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]
        steps = [0] * len(self.named)
        for i, (name, p) in enumerate(self.named):
            st = sd["state"].get(i, sd["state"].get(str(i)))
            if st is None:
                continue
            self.exp_avg[i].copy_(st["exp_avg"])
            self.exp_avg_sq[i].copy_(st["exp_avg_sq"])
            steps[i] = int(float(st["step"]))
        if any(steps):
            self.step_count = max(steps)
        self._steps_dev.copy_(torch.tensor(steps, dtype=torch.int32))

    def total_norm(self) -> Tensor:
        """sqrt(sum of squared group norms) (mhc_trainer.py:383), a device scalar."""
        return self.norms.pow(2).sum().sqrt()


SEED_STRIDE = 0x2545F491        # dropout seed-offset advance per step (odd: all 2^32 offsets visited)


class HVTrainer:
    """One training step = forward (train mode) + YOLOLoss + backward + all-reduce + clip + AdamW.

    graph=True (single process, HIP device): the whole step -- forward, loss, backward, gradient
    flush, clipping and AdamW -- is captured ONCE into a hipGraph (torch.cuda.CUDAGraph) and
    replayed every later step: ~3,000 kernel launches per step at 640^2 leave the host (an eager
    step spends ~90 ms issuing them).  The first step runs eagerly (it populates the caching
    allocator, the device tables and the optimizer's table), the second captures and replays.
    Dropout stays random per step: every dropout kernel adds the device word `seed_offset` to its
    seed, and the graph advances that word at its start.  Steps that run the stability monitor
    (every `monitor_every`-th, metrics only) run eagerly.  Inputs are copied into the graph's
    static buffers; the returned loss tensors are the graph's static outputs (overwritten by the
    next step).  A change of parameter storage or input shape re-captures."""

    def __init__(self, model, lr: float = 1e-3, weight_decay: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 max_grad_norm: float = 1.0, mhc_max_norm: float = 0.5, bucket_mb: int = 64,
                 broadcast_buffers: bool = True, group=None, monitor_every: int = 50, graph: bool = False,
                 manifold_weight: float = 0.0):
        self.model = model
        # the reference trainer's manifold regularisation term (mhc_trainer.py:248-255,299-340;
        # its default weight 0.01): off by default -- the committed reference never runs it (D10)
        if manifold_weight > 0:
            if graph:
                raise ValueError("manifold_weight > 0 (torch.linalg.eigvalsh) is not graph-capturable; use graph=False")
            model.hv_manifold_weight = float(manifold_weight)
        # _monitor_stability (eigvalsh of every H_res, signal ratios) is metrics-only: run it
        # every `monitor_every` steps instead of every forward (0 disables it)
        from .manifold import ManifoldHyperConnection
        self._mhc = [m for m in model.modules() if isinstance(m, ManifoldHyperConnection)]
        self.monitor_every = monitor_every
        self._set_monitor(monitor_every)
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        dev0 = named[0][1].device
        # ONE stream for every step, eager or captured: the gradient hooks keep each parameter's
        # AccumulateGrad node alive, and autograd runs that node (with the bucket flush hooked to
        # it) on the stream that was current when the node was created.  Created on the default
        # stream, a captured backward (on the capture stream) ran those accumulations and
        # flushes on the default stream -- outside the graph -- and replays lost them (torch's
        # "AccumulateGrad node's stream does not match" warning).  Hooks registered, eager steps
        # run and the graph captured on self.stream: the nodes' stream is the capture stream.
        self.stream = torch.cuda.Stream(device=dev0) if dev0.type == "cuda" else None
        with self._on_stream():
            self.grads = GradBuckets(named, bucket_mb << 20, group)
        self.opt = FusedAdamW(named, lr, weight_decay, betas, eps, (mhc_max_norm, max_grad_norm))
        self.world = self.grads.world
        self.group = group
        # DDP averaging.  Power-of-two worlds: the loss is scaled by 1/world before the backward
        # (exact: a power-of-two scale commutes with every rounding), so the bucket all-reduces
        # sum with no division pass over the gradients.  Other worlds: each bucket is divided by
        # the world right before its all-reduce, as torch DDP's allreduce hook does (a 1/3 loss
        # scale would round differently from DDP's averaging)
        self.grads.prescaled = self.world > 1 and (self.world & (self.world - 1)) == 0
        self.broadcast_buffers = broadcast_buffers and self.world > 1
        if self.world > 1:                         # DDP construction: replicas start identical
            self._broadcast(list(model.parameters()) + list(model.buffers()))
        self._buf_flats = self._flatten_buffers() if self.broadcast_buffers else []
        dev = named[0][1].device
        self.seed_offset = torch.zeros(1, dtype=torch.int32, device=dev)
        self.graph = bool(graph) and self.world == 1 and dev.type == "cuda"
        self.steps_done = 0
        self.replays = 0
        self.captures = 0
        self._g: Optional[Dict] = None

    def _on_stream(self):
        import contextlib
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _set_monitor(self, every: int, reset: bool = False) -> None:
        for m in self._mhc:
            m.monitor_every = every
            if reset:
                m._mon_count = 0

    def _flatten_buffers(self):
        """Rebind every buffer of the model as a view of one flat tensor per dtype, so the
        per-step DDP buffer broadcast (broadcast_buffers=True) is one collective per dtype
        with no packing or unpacking copies.  In-place updates (BN running statistics, mHC
        monitors) write through the views; load_state_dict copies into them."""
        by_dtype: Dict[torch.dtype, list] = {}
        for mod in self.model.modules():
            for name, b in mod._buffers.items():
                if b is not None:
                    by_dtype.setdefault(b.dtype, []).append((mod, name, b))
        flats = []
        self._buf_views = []
        for dt, entries in by_dtype.items():
            total = sum(b.numel() for _, _, b in entries)
            flat = torch.empty(total, device=entries[0][2].device, dtype=dt)
            off = 0
            with torch.no_grad():
                for mod, name, b in entries:
                    v = flat[off:off + b.numel()].view_as(b)
                    v.copy_(b)
                    mod._buffers[name] = v
                    self._buf_views.append((mod, name, v.data_ptr()))
                    off += b.numel()
            flats.append(flat)
        from .runtime import _bump_generation
        _bump_generation()                      # buffers were rebound: VersionWatch re-walks
        return flats

    def _broadcast(self, tensors):
        float_ts = [t for t in tensors if t.is_floating_point()]
        if float_ts:
            flat = torch.cat([t.detach().reshape(-1).float() for t in float_ts])
            dist.broadcast(flat, 0, group=self.group)
            off = 0
            with torch.no_grad():
                for t in float_ts:
                    t.copy_(flat[off:off + t.numel()].view_as(t))
                    off += t.numel()
        for t in tensors:
            if not t.is_floating_point():
                dist.broadcast(t, 0, group=self.group)

    def _buffers_still_flat(self) -> bool:
        """True while every buffer is still the view of the flat tensor it was bound to
        (model.to(), .float() or a buffer assignment rebinds buffers and would silently stop the
        per-step broadcast from reaching them)."""
        for mod, name, ptr in self._buf_views:
            b = mod._buffers.get(name)
            if b is None or b.data_ptr() != ptr:
                return False
        return True

    def _body(self, images: Tensor, targets: List[Tensor]) -> Dict[str, Tensor]:
        """zero -> forward -> loss -> backward -> flush/all-reduce -> clip + AdamW (all launches on
        the current stream; capturable at world 1)."""
        from .runtime import module_options, set_train_state
        set_train_state(module_options(self.model), self.seed_offset)
        try:
            self.seed_offset.add_(SEED_STRIDE)         # new dropout masks every step
            self.grads.zero()
            out = self.model(images, targets=targets, compute_loss=True)
            # detached (a captured step's: refreshed by every replay); holding the attached
            # outputs would keep this step's autograd graph alive into the next step
            self.last_predictions = {k: v.detach() for k, v in out.get("predictions", {}).items()}
            loss = out["loss"]
            total = loss["total_loss"]
            (total * (1.0 / self.world) if self.grads.prescaled else total).backward()
            self.grads.finish()
            self.opt.step(clip=True, active=self.grads.active_dev)
        finally:
            set_train_state()
        return loss

    def _eager(self, images: Tensor, targets: List[Tensor], monitor: bool) -> Dict[str, Tensor]:
        from .manifold import flush_stability
        if self.graph:                             # the graph never monitors; eager steps do on cadence
            self._set_monitor(1 if monitor else 0, reset=True)
        try:
            loss = self._body(images, targets)
        finally:
            if self.graph:
                self._set_monitor(0)
        flush_stability()                          # monitors' eigenvalue buffers current after every step
        return loss

    def _graph_key(self, images: Tensor, targets: List[Tensor]):
        """Everything a captured step bakes in: shapes, parameter storage, precision, the kernel
        variants (the model's HVOptions) and the clip norms the captured hv_grad_norms launch
        carries by value -- model.set_options() or new clip norms re-capture instead of replaying
        stale values.  lr / betas / eps / weight decay are NOT in it: AdamW reads them from the
        optimizer's device array, refreshed before every replay (FusedAdamW.sync_hyper), so a
        per-step scheduler keeps replaying the one captured graph."""
        from .runtime import module_options
        o = self.opt
        return (tuple(images.shape), images.dtype, tuple(tuple(t.shape) for t in targets),
                tuple(p.data_ptr() for p in self.grads.params), self.model.hv_precision
                if hasattr(self.model, "hv_precision") else None, module_options(self.model),
                tuple(float(m) for m in o.max_norms))

    def _capture(self, images: Tensor, targets: List[Tensor], key) -> None:
        from . import ops
        self._g = None
        torch.cuda.synchronize()
        static_x = images.detach().clone()
        static_t = [t.detach().clone() for t in targets]
        self._set_monitor(0)
        keep: List = []
        graph = torch.cuda.CUDAGraph()
        # thread_local: the autograd engine's worker thread issues the backward's launches onto
        # the capturing stream; the device-table uploads inside the step become graph memcpy
        # nodes whose pinned sources `keep` holds for the graph's lifetime
        steps = self.opt.step_count
        with ops.capture_keepalive(keep):
            with torch.cuda.graph(graph, stream=self.stream, capture_error_mode="thread_local"):
                loss = self._body(static_x, static_t)
        self.opt.step_count = steps            # the capture ran step()'s host side; no step happened
        self._g = {"graph": graph, "x": static_x, "t": static_t, "loss": loss, "keep": keep, "key": key}
        self.captures += 1

    def step(self, images: Tensor, targets: List[Tensor]) -> Dict[str, Tensor]:
        """One training step, issued on the trainer's stream (ordered after the caller's current
        stream's work, and the caller's stream waits for it before returning)."""
        if self.stream is None:
            return self._step(images, targets)
        cur = torch.cuda.current_stream(self.stream.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            loss = self._step(images, targets)
        cur.wait_stream(self.stream)
        for v in loss.values():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(cur)
        return loss

    def _step(self, images: Tensor, targets: List[Tensor]) -> Dict[str, Tensor]:
        self.model.train()
        if self._buf_flats and not self._buffers_still_flat():
            self._buf_flats = self._flatten_buffers()   # re-bind (the ranks do it in lock-step:
            # every rank sees the same module tree changes)
        for flat in self._buf_flats:               # DDP broadcast_buffers: rank 0's buffers
            dist.broadcast(flat, 0, group=self.group)
        monitor = self.monitor_every > 0 and self.steps_done % self.monitor_every == 0
        self.steps_done += 1
        if not self.graph:
            return self._eager(images, targets, monitor)
        key = self._graph_key(images, targets)
        if monitor or self.steps_done == 1:        # step 1 warms the allocator and the device tables
            return self._eager(images, targets, monitor)
        if self._g is None or self._g["key"] != key:
            self._capture(images, targets, key)
        g = self._g
        self.opt.sync_hyper()                      # this step's lr etc. into the array AdamW reads
        g["x"].copy_(images)
        for dst, src in zip(g["t"], targets):
            dst.copy_(src)
        g["graph"].replay()
        self.replays += 1
        self.opt.step_count += 1
        self.opt.bump_versions()                   # the replay's AdamW wrote the parameters
        return g["loss"]


def save_checkpoint(path: str, model, trainer: Optional["HVTrainer"] = None, epoch: int = 0, global_step: int = 0,
                    config: Optional[Dict] = None, history: Optional[Dict] = None,
                    best_val_loss: float = float("inf"), experiment_name: str = "hv_amd") -> None:
    """Checkpoint in the reference trainer's format (mhc_trainer.py:595-627): the same keys,
    model_state_dict in the reference parameter/buffer layout, optimizer_state_dict in
    torch.optim.AdamW layout (+ the reference optimizer's group keys), an empty scheduler state
    (LRScheduler.load_state_dict accepts it) and the state of an enabled GradScaler at its
    initial scale (the build uses no loss scaling: bf16 needs none), which
    GradScaler(enabled=True).load_state_dict accepts where an empty dict raises."""
    import time
    ck = {"epoch": epoch, "global_step": global_step, "model_state_dict": model.state_dict(),
          "optimizer_state_dict": trainer.opt.state_dict() if trainer is not None else {},
          "scheduler_state_dict": {},
          "scaler_state_dict": {"scale": 65536.0, "growth_factor": 2.0, "backoff_factor": 0.5,
                                "growth_interval": 2000, "_growth_tracker": 0}, "config": config or {}, "history": history or {},
          "best_val_loss": best_val_loss, "experiment_name": experiment_name, "timestamp": time.time()}
    torch.save(ck, path)


def load_checkpoint(path: str, model, trainer: Optional["HVTrainer"] = None, map_location=None) -> Dict:
    """mhc_trainer.py:629-656: loads model (and optimizer) state; tensors only (weights_only)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(ck["model_state_dict"])
    if trainer is not None and ck.get("optimizer_state_dict"):
        trainer.opt.load_state_dict(ck["optimizer_state_dict"])
    return ck
