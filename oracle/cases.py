"""Deterministic test-input recipes shared by the golden generator and the tests.

TEST INFRASTRUCTURE ONLY.  Inputs are regenerated from seeds so large-D fixtures need
not store them.
"""
from __future__ import annotations

import zlib

import torch

SK_CASES = [(8, 5), (8, 20), (32, 20), (64, 5), (64, 20), (128, 20), (256, 20), (512, 20),
            (1024, 20), (1792, 20)]
MHC_CASES = [(32, 4), (64, 4), (128, 4), (256, 4), (512, 4), (256, 2), (512, 2), (1024, 2),
             (1792, 2)]
MODEL_CASES = [  # (tag, tiny, family, size, batch, subsample rows of scale_0)
    ("tiny_wc_224_b2", True, "wc", 224, 2, 1),
    ("tiny_init_224_b2", True, "init", 224, 2, 1),
    ("base_wc_224_b2", False, "wc", 224, 2, 1),
    ("base_wc_512_b1", False, "wc", 512, 1, 4),
    ("base_wc_640_b1", False, "wc", 640, 1, 4),
]


def gen_seed(*key) -> torch.Generator:
    """Deterministic CPU generator keyed by a tuple of ints."""
    g = torch.Generator()
    g.manual_seed(zlib.crc32(repr(tuple(int(k) for k in key)).encode()) & 0x7FFFFFFF)
    return g


def sinkhorn_raw(D: int, iters: int, family: str) -> torch.Tensor:
    """Raw Sinkhorn input: N(0,1) (wc) or N(0, 0.01^2) (init-like)."""
    g = gen_seed(D, iters, 1 if family == "wc" else 2)
    return torch.randn(D, D, generator=g) * (1.0 if family == "wc" else 0.01)


def sinkhorn_cotangent(D: int, iters: int) -> torch.Tensor:
    return torch.randn(D, D, generator=gen_seed(D, iters, 3))


def mhc_input(D: int, e: int) -> torch.Tensor:
    return torch.randn(64, D, generator=gen_seed(D, e, 11))


def mhc_cotangent(D: int, e: int) -> torch.Tensor:
    return torch.randn(64, D, generator=gen_seed(D, e, 12))


def model_input(B: int, S: int) -> torch.Tensor:
    return torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1))
