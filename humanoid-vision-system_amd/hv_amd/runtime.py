"""Forward-scoped runtime state: compute precision and per-forward prepared coefficients.

The reference recomputes every parameter-only quantity (sigmoid gates, the Sinkhorn
projection, autocast weight copies) inside every forward.  Here the top-level module
prepares all of them once at the start of a forward (prep.PrepProgram: a fixed handful of
grouped launches for all 76 mHC sites and every Conv/Linear weight) and the layers look
them up by module.  With
``freeze()`` (eval streaming) the prepared state is reused across forwards until a
parameter's version counter changes.
"""
from __future__ import annotations

import contextvars
import dataclasses
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

_CTX: contextvars.ContextVar = contextvars.ContextVar("hv_runtime_ctx", default=None)

PRECISIONS = {"bf16": torch.bfloat16, "fp32": torch.float32}


@dataclass(frozen=True)
class HVOptions:
    """Per-model execution options: kernel selection and the exact restructurings of the
    inference path.  A model (or a standalone layer) carries one in ``hv_options``; every forward
    copies it into its RunCtx, so the options are per model and per call -- there is no
    process-global switch, and concurrent forwards (AsyncInferenceEngine's workers, other
    streams) never see each other's choice.  The defaults are the product configuration."""
    use_fused_mhc: bool = True        # one-launch mHC kernel for D <= 128 (hv_mhc_fused)
    fold_max_d: int = 1024            # fold H_pre into W1 for D <= this
    cls_only_last_block: bool = True  # last ViT block on the CLS query only (exact)
    group_qkv: bool = True            # q / k / v GEMM1 as one N = 3*2Hd GEMM (exact)
    parallel_qkv: bool = False        # q / k / v on three streams: measured slower (tools/ab_vit.py)
    prep_overlap: bool = False        # Sinkhorn + mHC prep on a side stream at every batch
    prep_overlap_min_batch: int = 1   # ... and from this batch on (B=16: -0.9..-1.8 %; B=1 recompute: -3 % on
                                      # the closing build, +0.7 % before the 32x64 tile; profiles/r06/prep_overlap_b1_recompute_ab.txt)
    direct_stem: bool = True          # MFMA stem conv straight from the NCHW image (hv_conv_stem)
    splitk: bool = False              # split-K for small output grids: measured no gain
    splitk_small_m: int = 0           # ... but for GEMMs of at most this many rows (the 16-row final fusion)
    gemm_variant: int = 0             # hv_gemm_desc.variant for every GEMM (HV_GV_*), 0 = automatic
    mhc_variant: int = 0              # hv_mhc_fused_args.variant (HV_MV_*), 0 = automatic
    wgrad_variant: int = 0            # hv_wgrad_desc.variant for the weight gradients (HV_WV_*), 0 = automatic
    mhc256_min_tokens: int = 25600    # D = 256 sites fused (split-hidden) from this many tokens (ops._mhc_variant)
    mhc_tok: bool = True              # token-tile fused kernel for small-T sites (HV_MV_TOK, ops._mhc_variant)
    mhc_tok_split: bool = True        # ... with a tile's hidden units split over 2 / 4 workgroups when tiles < CUs
    branch_min_batch: int = 8         # independent branches on side streams from this batch (Branches)

    def replace(self, **kw) -> "HVOptions":
        return dataclasses.replace(self, **kw)


DEFAULT_OPTIONS = HVOptions()


def module_options(module: torch.nn.Module) -> HVOptions:
    o = getattr(module, "hv_options", None)
    return o if isinstance(o, HVOptions) else DEFAULT_OPTIONS


@dataclass
class RunCtx:
    dtype: torch.dtype
    opts: HVOptions = DEFAULT_OPTIONS
    plans: Dict[int, object] = field(default_factory=dict)
    program: Optional[object] = None      # prep.PrepProgram that produced `plans` (grouped prep)
    prep_event: Optional[object] = None   # side-stream prep not yet joined (PrepProgram.run overlap)

    def join_prep(self) -> None:
        """Make the current stream wait for the side-stream Sinkhorn + mHC prep (once)."""
        ev = self.prep_event
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
            self.prep_event = None


def current() -> Optional[RunCtx]:
    return _CTX.get()


class Branches:
    """Independent parts of one eval forward on side streams: the three detection heads (each
    starts as soon as the pyramid has produced its scale) and the small / medium scale
    enhancements of the backbone beside stages 3-4.  Their launches leave CUs idle in their tails
    (and the 20x20 heads use tens of workgroups), so overlapping parts that share no data fills
    the chip better.  fork(fn) runs fn on a side stream that first waits for everything issued so
    far on the forward's stream; join() makes the forward's stream wait for every forked branch.
    Results of a branch may be read on the forward's stream only after join().  Side streams are
    kept per (device, forward stream), so concurrent forwards on different streams never share
    one; a graph captured over the forward records each fork / join as graph edges.
    Disabled (fork = call), the forward is the single-stream one."""
    _STREAMS: Dict[tuple, list] = {}

    def __init__(self, enabled: bool):
        self.main = torch.cuda.current_stream() if enabled else None
        self.pending: list = []
        self.used = 0

    def _side(self) -> "torch.cuda.Stream":
        key = (self.main.device.index, self.main.cuda_stream)
        pool = Branches._STREAMS.setdefault(key, [])
        if self.used == len(pool):
            pool.append(torch.cuda.Stream(device=self.main.device))
        s = pool[self.used]
        self.used += 1
        return s

    def fork(self, fn):
        if self.main is None:
            return fn()
        s = self._side()
        s.wait_stream(self.main)
        with torch.cuda.stream(s):
            out = fn()
            done = torch.cuda.Event()
            done.record(s)
        self.pending.append(done)
        return out

    def join(self) -> None:
        for ev in self.pending:
            self.main.wait_event(ev)
        self.pending.clear()
        self.used = 0           # the side streams' later work is ordered after this join


class _TrainState:
    """Process-level state of the training step in progress (train_model.system_forward sets it,
    HVTrainer clears it after the step).  Training forwards enter no RunCtx, and autograd runs
    their backward on its own worker thread, where a ContextVar set by the forward is not
    visible -- so the model's HVOptions and the dropout seed-offset word of a training step live
    here, read by the forward and the backward launches alike.  One training step at a time per
    process (the trainer's contract)."""
    opts: HVOptions = DEFAULT_OPTIONS
    seed_offset: Optional[torch.Tensor] = None      # device int32 [1] (hv_kernels.h seed_offset)


_TRAIN = _TrainState()


def set_train_state(opts: Optional[HVOptions] = None, seed_offset: Optional[torch.Tensor] = None) -> None:
    _TRAIN.opts = opts if opts is not None else DEFAULT_OPTIONS
    _TRAIN.seed_offset = seed_offset


def carry_train_state(namespace: dict) -> None:
    """Every torch.autograd.Function class in `namespace` (a module's globals()) records the
    training state of its forward (the model's HVOptions, the dropout seed-offset word) and runs
    its backward under that state, so the backward -- on autograd's worker thread, after
    system_forward has returned and restored _TRAIN -- launches with the forward's kernel variants
    and seeds, and no model's options outlive its forward in the process-level _TRAIN."""
    for cls in list(namespace.values()):
        if not (isinstance(cls, type) and issubclass(cls, torch.autograd.Function)) or cls is torch.autograd.Function:
            continue
        if getattr(cls, "_hv_carries_state", False):
            continue
        fwd, bwd = cls.forward, cls.backward

        def forward(ctx, *a, _fwd=fwd, **k):
            ctx.hv_train_state = (_TRAIN.opts, _TRAIN.seed_offset)
            return _fwd(ctx, *a, **k)

        def backward(ctx, *g, _bwd=bwd):
            st = getattr(ctx, "hv_train_state", None)
            if st is None:
                return _bwd(ctx, *g)
            prev = (_TRAIN.opts, _TRAIN.seed_offset)
            _TRAIN.opts, _TRAIN.seed_offset = st
            try:
                return _bwd(ctx, *g)
            finally:
                _TRAIN.opts, _TRAIN.seed_offset = prev

        cls.forward, cls.backward = staticmethod(forward), staticmethod(backward)
        cls._hv_carries_state = True


def seed_offset_ptr() -> Optional[int]:
    """Device pointer of the current training step's dropout seed offset (None: seeds by value)."""
    t = _TRAIN.seed_offset
    return None if t is None else t.data_ptr()


def options() -> HVOptions:
    """The options of the forward in progress: its RunCtx's, else the training step's (set by
    system_forward for the forward and its backward), else the defaults."""
    ctx = _CTX.get()
    return ctx.opts if ctx is not None else _TRAIN.opts


class use_ctx:
    def __init__(self, ctx: RunCtx):
        self.ctx = ctx
        self.tok = None

    def __enter__(self):
        self.tok = _CTX.set(self.ctx)
        return self.ctx

    def __exit__(self, *exc):
        _CTX.reset(self.tok)
        return False


def resolve_dtype(module: torch.nn.Module) -> torch.dtype:
    ctx = current()
    if ctx is not None:
        return ctx.dtype
    return PRECISIONS[getattr(module, "hv_precision", "bf16")]


def require_cuda(x: torch.Tensor, what: str) -> None:
    if not x.is_cuda:
        raise RuntimeError(f"{what}: hv_amd runs on the MI355X HIP path only (got a {x.device} tensor); "
                           "move the model and inputs to 'cuda'")


def param_versions(module: torch.nn.Module):
    return tuple((p.data_ptr(), p._version) for p in module.parameters())


# Any parameter / buffer / submodule (re)registration anywhere bumps this generation, so a
# VersionWatch re-walks its module tree only when the tree may have changed (the walk costs
# ~2.6 ms on the base model; the per-call snapshot ~0.4 ms).
_REG_GEN = [0]


def _bump_generation(*_args):
    _REG_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_generation)
torch.nn.modules.module.register_module_buffer_registration_hook(_bump_generation)
torch.nn.modules.module.register_module_module_registration_hook(_bump_generation)


# buffers the forward itself writes (mHC monitors, Sinkhorn history): not inputs of the forward
_OUTPUT_BUFFERS = ("convergence_history", "eigenvalues", "signal_ratio_history", "gradient_norms")


class VersionWatch:
    """Cheap change detector for everything a prepared / captured forward baked in: the
    storage pointer and in-place version counter of every parameter and input buffer (BN
    statistics, anchors, ...) of `module`, and the storage pointer of every buffer the forward
    WRITES (Sinkhorn histories, monitor buffers: a captured graph keeps writing into the
    storage it saw at capture).  In-place updates (optimizer steps, load_state_dict copies),
    `.data` swaps, buffer rebinding (`module.buf = t`, `_buffers[...] = t` as `.to()` does,
    HVTrainer's flat-buffer views) and `.to()` moves all change the snapshot.

    Buffers are looked up by (module, name) on every call -- `.to()` / `.float()` replace the
    buffer tensor objects without a registration hook, so holding the tensors would miss them."""

    def __init__(self, module: torch.nn.Module):
        self.module = module
        self._gen = -1
        self._params = []
        self._ins = []
        self._outs = []

    def snapshot(self):
        if self._gen != _REG_GEN[0]:
            self._params = list(self.module.parameters())
            self._ins, self._outs = [], []
            for mname, mod in self.module.named_modules():
                for bname in mod._buffers:
                    (self._outs if bname in _OUTPUT_BUFFERS else self._ins).append((mod._buffers, bname))
            self._gen = _REG_GEN[0]
        ps = self._params
        ins = [d.get(n) for d, n in self._ins]
        ins = [b for b in ins if b is not None]
        outs = [d.get(n) for d, n in self._outs]
        return (tuple([t._version for t in ps]), tuple([t.data_ptr() for t in ps]),
                tuple([t._version for t in ins]), tuple([t.data_ptr() for t in ins]),
                tuple([0 if t is None else t.data_ptr() for t in outs]))
