"""S8: CUDA-autocast (bf16) op policy, emulated on CPU -- TEST INFRASTRUCTURE ONLY.

The reference's mixed-precision contract is CUDA autocast: `torch.cuda.amp.autocast(dtype=bf16)`
inside every ManifoldHyperConnection.forward (src/models/manifold_layers.py:186,248) and around
the whole training forward (src/training/mhc_trainer.py:241, dtype bfloat16 from
configs/training.yaml:134 / src/config/base_config.py:233-238).  On CPU `torch.cuda.amp.autocast`
is a no-op, and CPU `torch.autocast` follows a different op list (it keeps layer_norm in bf16),
so the reference's OWN bf16 numerics cannot be produced by running it on this container as is.

`CudaAutocastBF16` is a TorchFunctionMode that applies CUDA autocast's per-op policy at the
Python op boundary (above autograd, like autocast itself, so the casts are recorded and the
backward runs in the dtypes the forward produced):
  * lower-precision ops (CUDA autocast "lower_precision_fp" list: convolutions, linear, matmul,
    mm, bmm, addmm, baddbmm, einsum ...): fp32 floating inputs are cast to bf16, the op runs in
    bf16 (fp32 accumulation inside the CPU GEMM, bf16 output) -- as cuBLAS/MIOpen do;
  * fp32 ops (the "fp32" and "fp32_set_opt_dtype" lists: layer_norm, group_norm, softmax,
    log_softmax, exp, log, pow, rsqrt, reciprocal, sum, prod, cumsum, mse_loss,
    binary_cross_entropy_with_logits, norm ...): bf16 inputs are cast to fp32;
  * everything else runs in the dtype of its inputs (elementwise activations, BatchNorm,
    pooling, adds -- with torch's usual bf16/fp32 type promotion).
Sinkhorn (softmax, sums and divisions of fp32 parameters) therefore stays fp32, exactly as on the
GPU.  Used only by oracle/gen_golden.py to write the *_bf16ref fixtures; never by the product.
"""
from __future__ import annotations

import torch
from torch.overrides import TorchFunctionMode

LOWER = {"conv1d", "conv2d", "conv3d", "conv_transpose1d", "conv_transpose2d", "conv_transpose3d",
         "convolution", "_convolution", "linear", "matmul", "__matmul__", "__rmatmul__", "mm", "mv", "bmm",
         "addmm", "addmv", "addr", "addbmm", "baddbmm", "einsum", "chain_matmul", "prelu",
         "scaled_dot_product_attention"}
FP32 = {"layer_norm", "native_layer_norm", "group_norm", "softmax", "log_softmax", "exp", "expm1", "log",
        "log10", "log2", "log1p", "pow", "__pow__", "__rpow__", "rsqrt", "reciprocal", "softplus", "sum", "prod",
        "cumsum", "cumprod", "logsumexp", "norm", "frobenius_norm", "cdist", "dist", "renorm", "mse_loss",
        "l1_loss", "smooth_l1_loss", "huber_loss", "binary_cross_entropy_with_logits", "nll_loss", "kl_div",
        "cosine_similarity", "acos", "asin", "cosh", "sinh", "tan", "erfinv"}


def _cast(x, src, dst):
    if isinstance(x, torch.Tensor):
        return x.to(dst) if x.dtype == src else x
    if isinstance(x, (list, tuple)):
        return type(x)(_cast(v, src, dst) for v in x)
    return x


class CudaAutocastBF16(TorchFunctionMode):
    """`with CudaAutocastBF16(): model(x)` runs `model` under CUDA autocast's bf16 policy."""

    def __init__(self):
        super().__init__()
        self.counts = {"lower": 0, "fp32": 0}

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = getattr(func, "__name__", "")
        if name in LOWER:
            self.counts["lower"] += 1
            args = _cast(args, torch.float32, torch.bfloat16)
            kwargs = {k: _cast(v, torch.float32, torch.bfloat16) for k, v in kwargs.items()}
        elif name in FP32 and kwargs.get("dtype") is None:
            self.counts["fp32"] += 1
            args = _cast(args, torch.bfloat16, torch.float32)
            kwargs = {k: _cast(v, torch.bfloat16, torch.float32) for k, v in kwargs.items()}
        return func(*args, **kwargs)


class MhcOnly:
    """Scope the policy to the reference's own autocast region: the body of
    ManifoldHyperConnection.forward (manifold_layers.py:247-263); constrained_matrices (Sinkhorn,
    sigmoids) runs before it in fp32 either way."""

    def __init__(self, ml):
        self.ml = ml
        self.orig = None

    def __enter__(self):
        ml = self.ml
        self.orig = orig = ml.ManifoldHyperConnection.forward

        def fwd(mod, x):
            with CudaAutocastBF16():
                return orig(mod, x)
        ml.ManifoldHyperConnection.forward = fwd
        return self

    def __exit__(self, *exc):
        self.ml.ManifoldHyperConnection.forward = self.orig
        return False
