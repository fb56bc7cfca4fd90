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
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

_CTX: contextvars.ContextVar = contextvars.ContextVar("hv_runtime_ctx", default=None)

PRECISIONS = {"bf16": torch.bfloat16, "fp32": torch.float32}


@dataclass
class RunCtx:
    dtype: torch.dtype
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
    statistics, anchors, ...) of `module`.  In-place updates (optimizer steps, load_state_dict
    copies), `.data` swaps and `.to()` moves all change the snapshot."""

    def __init__(self, module: torch.nn.Module):
        self.module = module
        self._gen = -1
        self._ts = []

    def snapshot(self):
        if self._gen != _REG_GEN[0]:
            self._ts = list(self.module.parameters()) + [
                b for n, b in self.module.named_buffers() if not n.endswith(_OUTPUT_BUFFERS)]
            self._gen = _REG_GEN[0]
        ts = self._ts
        return tuple([t._version for t in ts]), tuple([t.data_ptr() for t in ts])
