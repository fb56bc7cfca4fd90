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
