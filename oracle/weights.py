"""Deterministic weight formula shared by the golden generator and the parity tests.

TEST INFRASTRUCTURE ONLY: imported by ``oracle/gen_golden.py``, ``tests/`` and
``__graft_entry__.smoke()``; never by the product path.

Weights are regenerated from (parameter name, shape, family) instead of being stored,
so full-model fixtures stay small (the base model is 353.8M parameters).  Each tensor
is drawn from torch's CPU mt19937 generator seeded with ``crc32(family + name)``; the
same torch build runs in this container and on the GPU box, so both sides regenerate
bit-identical tensors.

Families:
* ``init`` -- the reference's own init scales (``manifold_layers.py:191-203``,
  ``vision_backbone.py:90-97``, ``hybrid_vision.py:183-197``): the ill-conditioned
  regime (H_pre ~ 0.5, H_res ~ 1/D, MLP weights N(0, 0.01)).
* ``wc`` -- "well-conditioned": spread mHC coefficients, xavier-scale MLP weights,
  perturbed BN / LN / RMSNorm affine parameters, wider prediction-conv weights so
  class margins are wide.
Uniform draws with the target standard deviation replace the reference's normal draws.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import torch

SQRT3 = math.sqrt(3.0)

# Buffers that are state, not weights: left exactly as the module built them.
_KEEP_BUFFERS = (
    "convergence_history", "gradient_norms", "eigenvalues", "signal_ratio_history",
    "num_batches_tracked", "anchors",
)


def _gen(family: str, name: str) -> torch.Generator:
    g = torch.Generator(device="cpu")
    g.manual_seed(zlib.crc32(f"{family}:{name}".encode()) & 0x7FFFFFFF)
    return g


def _uniform(shape, std: float, g: torch.Generator, center: float = 0.0) -> torch.Tensor:
    a = std * SQRT3
    return (torch.rand(shape, generator=g, dtype=torch.float32) * 2.0 - 1.0) * a + center


def make_tensor(name: str, shape: Tuple[int, ...], family: str = "init") -> torch.Tensor | None:
    """Return the formula value for one state_dict entry (None = keep the module's own)."""
    if name.split(".")[-1] in _KEEP_BUFFERS:
        return None
    g = _gen(family, name)
    leaf = name.split(".")[-1]
    name = "." + name  # so ".bn." style matches also hit root-level modules
    wc = family == "wc"
    shape = tuple(shape)

    # --- mHC coefficient matrices (manifold_layers.py:149-157,194-196) ---
    if leaf in ("H_pre_raw", "H_post_raw", "H_res_raw"):
        if wc:
            return _uniform(shape, 1.2, g)
        a = 0.1 * math.sqrt(6.0 / (shape[0] + shape[1]))
        return _uniform(shape, a / SQRT3, g)

    is_bn = (".bn." in name or ".conv_layers.1." in name or ".conv_layers.4." in name
             or (".refinement_convs." in name and name.split(".")[-2] in ("1", "4")))
    if is_bn:
        if leaf == "weight":
            return _uniform(shape, 0.15 if wc else 0.02, g, center=1.0)
        if leaf == "bias":
            return _uniform(shape, 0.1 if wc else 0.01, g)
        if leaf == "running_mean":
            return _uniform(shape, 0.1 if wc else 0.01, g)
        if leaf == "running_var":
            return _uniform(shape, 0.15 if wc else 0.02, g, center=1.0).abs() + 0.05
    if ".norm_pre." in name or ".norm_post." in name:
        if leaf == "weight":
            return _uniform(shape, 0.2 if wc else 0.0, g, center=1.0)
        return _uniform(shape, 0.1 if wc else 0.0, g)
    if leaf == "scale":  # RMSNorm (manifold_layers.py:446)
        return _uniform(shape, 0.2 if wc else 0.0, g, center=1.0)
    if leaf in ("pos_embed", "position_embeddings", "cls_token"):
        return _uniform(shape, 0.02 if not wc else 0.2, g)

    if leaf == "weight" and len(shape) == 4:  # conv (kaiming fan_out, hybrid_vision.py:186-190)
        fan_out = shape[0] * shape[2] * shape[3]
        std = math.sqrt(2.0 / fan_out)
        if wc and ".pred_conv." in name:
            std = 0.1
        elif wc:
            std = math.sqrt(2.0 / (shape[1] * shape[2] * shape[3]))
        return _uniform(shape, std, g)
    if leaf == "weight" and len(shape) == 2:  # nn.Linear (hybrid_vision.py:194-197)
        std = math.sqrt(2.0 / (shape[0] + shape[1])) if wc else 0.01
        return _uniform(shape, std, g)
    if leaf == "bias":
        return _uniform(shape, 0.05 if wc else 0.01, g)
    raise KeyError(f"no weight rule for {name} {shape}")


def fill_state_dict(sd: Dict[str, torch.Tensor], family: str = "init") -> Dict[str, torch.Tensor]:
    """Return a copy of ``sd`` with every weight replaced by the formula value."""
    out = {}
    for k, v in sd.items():
        t = make_tensor(k, tuple(v.shape), family)
        out[k] = v.clone() if t is None else t.to(v.dtype)
    return out


def load_formula_weights(module: torch.nn.Module, family: str = "init") -> None:
    """In-place: overwrite a module's parameters/buffers with the formula values."""
    sd = module.state_dict()
    module.load_state_dict(fill_state_dict(sd, family))


def iter_formula(names_shapes: Iterable[Tuple[str, Tuple[int, ...]]], family: str = "init"):
    for n, s in names_shapes:
        yield n, make_tensor(n, s, family)
