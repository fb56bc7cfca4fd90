"""CNN backbone on the HIP path (reference src/models/vision_backbone.py).

Activations stay NHWC end to end: the conv output is already the token-major [B*H*W, C]
matrix the mHC layer consumes, so the reference's permute/reshape round trips
(vision_backbone.py:121-123, 371-391) disappear.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import ops
from .layers import conv_prep, ctx_scope, run_conv, to_nchw_view, to_nhwc
from .manifold import ManifoldHyperConnection
from .runtime import Branches, current, options, require_cuda, resolve_dtype

# Direct stem conv (hv_conv_stem: bf16 = LDS-staged input tile + one MFMA k-step per 16 pixels)
# instead of the NCHW->NHWC pass + implicit GEMM (237 us at B=16 640^2).  Same-box A/B
# (profiles/r02/stem_direct_ab.txt): 759.5 vs 749.9 img/s, B=1 frozen p50 5.335 vs 5.363 ms.
# HVOptions(direct_stem=False) restores the GEMM path.


class ConvMHCLayer(nn.Module):
    """vision_backbone.py:10-134: conv -> BN -> act -> mHC(C_out) -> SE gate -> (+x)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int = 3, stride: int = 1,
                 padding: Optional[int] = None, groups: int = 1, expansion_rate: int = 4,
                 use_mhc: bool = True, activation: str = "silu", sk_iterations: int = 20):
        super().__init__()
        if groups != 1:
            raise NotImplementedError("grouped convolution is not on the HybridVision path")
        self.in_channels, self.out_channels, self.stride, self.use_mhc = in_channels, out_channels, stride, use_mhc
        padding = kernel_size // 2 if padding is None else padding
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False)
        self.bn = nn.BatchNorm2d(out_channels)
        acts = {"silu": nn.SiLU(), "relu": nn.ReLU(inplace=True), "gelu": nn.GELU()}
        if activation not in acts:
            raise ValueError(f"Unsupported activation: {activation}")
        self.activation = acts[activation]
        self.act_name = activation
        self.mhc = ManifoldHyperConnection(out_channels, expansion_rate=expansion_rate,
                                           sk_iterations=sk_iterations) if use_mhc else None
        self.use_residual = in_channels == out_channels and stride == 1
        if use_mhc and out_channels >= 32:
            self.channel_attention = nn.Sequential(
                nn.AdaptiveAvgPool2d(1), nn.Conv2d(out_channels, out_channels // 4, 1), self.activation,
                nn.Conv2d(out_channels // 4, out_channels, 1), nn.Sigmoid())
        else:
            self.channel_attention = None
        nn.init.kaiming_normal_(self.conv.weight, mode="fan_out", nonlinearity="relu")
        nn.init.ones_(self.bn.weight)
        nn.init.zeros_(self.bn.bias)

    def forward_nhwc(self, x: torch.Tensor, extra_residual: Optional[torch.Tensor] = None,
                     pool: bool = False) -> torch.Tensor:
        """pool=True appends the stem's MaxPool2d(2, 2) (vision_backbone.py:248); with a gate and
        no residual the gate multiply and the pool are one pass (ops.maxpool2x2(y, gate))."""
        if pool:
            if self.channel_attention is not None and not self.use_residual and extra_residual is None:
                return self._forward_gated(x, pool=True)
            return ops.maxpool2x2(self.forward_nhwc(x, extra_residual))
        y = run_conv(x, self.conv, self.bn, self.act_name, self)
        return self._after_conv(x, y, extra_residual)

    def forward_image(self, img: torch.Tensor, dtype: torch.dtype, nhwc: bool = False) -> Optional[torch.Tensor]:
        """First backbone layer straight from the image (NCHW fp32, or NHWC `dtype`): the direct
        stem conv (ops.conv_stem) replaces the NCHW->NHWC pass + implicit GEMM.  None if not
        applicable."""
        if self.use_residual:
            return None
        w, s, b = conv_prep(self.conv, self.bn, dtype, self)
        y = ops.conv_stem(img, w, self.conv.kernel_size[0], self.conv.stride[0], self.conv.padding[0], dtype,
                          scale=s, bias=b, act=self.act_name, nhwc=nhwc)
        return None if y is None else self._after_conv(None, y, None)

    def _after_conv(self, x, y, extra_residual):
        if self.mhc is not None:
            n, h, w, c = y.shape
            y = self.mhc.forward_tokens(y.view(-1, c)).view(n, h, w, c)
            if self.channel_attention is not None:
                ca = self.channel_attention
                gate = ops.se_gate(y, ca[1].weight, ca[1].bias, ca[3].weight, ca[3].bias)
                y = ops.scale_residual(y, gate, x if self.use_residual else None)
                if extra_residual is not None:
                    y = ops.add_scaled(y, extra_residual, 1.0)
                return y
        if self.use_residual:
            y = ops.add_scaled(y, x, 1.0)
        if extra_residual is not None:
            y = ops.add_scaled(y, extra_residual, 1.0)
        return y

    def _forward_gated(self, x: torch.Tensor, pool: bool) -> torch.Tensor:
        y = run_conv(x, self.conv, self.bn, self.act_name, self)
        n, h, w, c = y.shape
        y = self.mhc.forward_tokens(y.view(-1, c)).view(n, h, w, c)
        ca = self.channel_attention
        gate = ops.se_gate(y, ca[1].weight, ca[1].bias, ca[3].weight, ca[3].bias)
        return ops.maxpool2x2(y, gate) if pool else ops.scale_residual(y, gate, None)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        require_cuda(x, "ConvMHCLayer")
        if self.training:
            from . import train_model as TM
            return to_nchw_view(TM.conv_mhc_layer(self, TM.nhwc_in(x, resolve_dtype(self)), TM.module_H(self)))
        with ctx_scope(self) as ctx:
            return to_nchw_view(self.forward_nhwc(to_nhwc(x, ctx.dtype)))


class ResidualMHCLayer(nn.Module):
    """vision_backbone.py:137-196 (bottleneck branch for channels >= 64)."""

    def __init__(self, channels: int, num_blocks: int = 2, expansion_rate: int = 4, bottleneck: bool = True,
                 sk_iterations: int = 20):
        super().__init__()
        self.channels, self.num_blocks = channels, num_blocks
        kw = dict(expansion_rate=expansion_rate, sk_iterations=sk_iterations)
        if bottleneck and channels >= 64:
            self.blocks = nn.Sequential(ConvMHCLayer(channels, channels // 2, kernel_size=1, **kw),
                                        ConvMHCLayer(channels // 2, channels, kernel_size=3, **kw))
            self.projection = ConvMHCLayer(channels, channels, kernel_size=1, **kw)
        else:
            self.blocks = nn.Sequential(*[ConvMHCLayer(channels, channels, kernel_size=3, **kw)
                                          for _ in range(num_blocks)])
            self.projection = nn.Identity()

    def forward_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        y = x
        for b in self.blocks:
            y = b.forward_nhwc(y)
        if isinstance(self.projection, nn.Identity):
            return ops.add_scaled(y, x, 1.0)
        return self.projection.forward_nhwc(y, extra_residual=x)

    def forward(self, x):
        require_cuda(x, "ResidualMHCLayer")
        if self.training:
            from . import train_model as TM
            return to_nchw_view(TM.residual_layer(self, TM.nhwc_in(x, resolve_dtype(self)), TM.module_H(self)))
        with ctx_scope(self) as ctx:
            return to_nchw_view(self.forward_nhwc(to_nhwc(x, ctx.dtype)))


class HybridVisionBackbone(nn.Module):
    """vision_backbone.py:199-413."""

    def __init__(self, input_channels: int = 3, base_channels: int = 32, num_blocks: List[int] = (2, 3, 4, 2),
                 use_mhc: bool = True, activation: str = "silu", dropout_rate: float = 0.1,
                 sk_iterations: int = 20, verbose: bool = True):
        super().__init__()
        self.input_channels, self.base_channels, self.use_mhc = input_channels, base_channels, use_mhc
        self.dropout_rate = dropout_rate
        kw = dict(use_mhc=use_mhc, activation=activation, sk_iterations=sk_iterations)
        self.stem = nn.Sequential(
            ConvMHCLayer(input_channels, base_channels, 3, 2, 1, **kw),
            ConvMHCLayer(base_channels, base_channels, 3, 1, 1, **kw),
            ConvMHCLayer(base_channels, base_channels * 2, 3, 1, 1, **kw),
            nn.MaxPool2d(kernel_size=2, stride=2))
        cur = base_channels * 2
        stage_channels = [cur, cur * 2, cur * 4, cur * 8]
        self.stages = nn.ModuleList()
        for i, (nl, co) in enumerate(zip(num_blocks, stage_channels)):
            layers = [ConvMHCLayer(cur, co, kernel_size=3, stride=2 if i > 0 else 1, **kw)]
            layers += [ResidualMHCLayer(co, num_blocks=2, expansion_rate=4, bottleneck=True,
                                        sk_iterations=sk_iterations) for _ in range(1, nl)]
            self.stages.append(nn.Sequential(*layers))
            cur = co
        mk = (lambda c: ManifoldHyperConnection(c, expansion_rate=4, sk_iterations=sk_iterations)) if use_mhc \
            else (lambda c: nn.Identity())
        self.enhance_large = mk(stage_channels[-1])
        self.enhance_medium = mk(stage_channels[-2])
        self.enhance_small = mk(stage_channels[-3])
        self.dropout = nn.Dropout2d(dropout_rate) if dropout_rate > 0 else nn.Identity()
        self.output_channels = {"stem": base_channels * 2, "stage_1": stage_channels[0],
                                "stage_2": stage_channels[1], "stage_3": stage_channels[2],
                                "stage_4": stage_channels[3]}
        self.stride_factors = {"stem": 4, "stage_1": 4, "stage_2": 8, "stage_3": 16, "stage_4": 32}
        if verbose:
            print(f"Backbone initialized with channels: {self.output_channels}")

    def forward_nhwc(self, x: Optional[torch.Tensor], image: Optional[torch.Tensor] = None,
                     branches: Optional[Branches] = None) -> Dict[str, torch.Tensor]:
        """x: NHWC input; or image: the NCHW fp32 batch, whose first conv then runs as the direct
        stem kernel (falls back to the NHWC conversion + implicit GEMM when not applicable)."""
        layers = list(self.stem)[:3]
        dt = current().dtype
        if image is not None and not options().direct_stem:
            x, image = to_nhwc(image, dt), None
        if image is not None:
            y = layers[0].forward_image(image, dt)
            if y is None:
                y = layers[0].forward_nhwc(to_nhwc(image, dt))
            x, layers = y, layers[1:]
        else:
            # NHWC input (the engine's preprocessed frame): the same direct stem kernel, so both
            # input layouts give identical results
            y = layers[0].forward_image(x, dt, nhwc=True) if x.shape[-1] == 3 and options().direct_stem else None
            if y is not None:
                x, layers = y, layers[1:]
        for i, lyr in enumerate(layers):
            x = lyr.forward_nhwc(x, pool=lyr is self.stem[2])     # stem[3] MaxPool2d fused into stem[2]
        raw = {"stem": x}

        def enh(mod, f):
            if isinstance(mod, nn.Identity):
                return f
            n, h, w, c = f.shape
            return mod.forward_tokens(f.view(-1, c)).view(n, h, w, c)

        # the small / medium scale enhancements read stage outputs the later stages only read too:
        # with branches they run on side streams beside stages 3-4 (joined before returning)
        br = branches if branches is not None else Branches(False)
        out = {}
        for i, st in enumerate(self.stages):
            for lyr in st:
                x = lyr.forward_nhwc(x)
            raw[f"stage_{i + 1}"] = x
            if i == 1:
                out["scale_small"] = br.fork(lambda f=x: enh(self.enhance_small, f))
            elif i == 2:
                out["scale_medium"] = br.fork(lambda f=x: enh(self.enhance_medium, f))
        out["scale_large"] = enh(self.enhance_large, raw["stage_4"])
        br.join()
        out["raw_features"] = raw
        return out

    def forward(self, x: torch.Tensor) -> Dict[str, torch.Tensor]:
        require_cuda(x, "HybridVisionBackbone")
        if self.training:
            from . import train_model as TM
            out = TM.backbone(self, TM.nhwc_in(x, resolve_dtype(self)), TM.module_H(self))
        else:
            with ctx_scope(self) as ctx:
                out = self.forward_nhwc(to_nhwc(x, ctx.dtype))
        res = {k: to_nchw_view(v) for k, v in out.items() if k != "raw_features"}
        res["raw_features"] = {k: to_nchw_view(v) for k, v in out["raw_features"].items()}
        return res

    def get_output_channels(self) -> Dict[str, int]:
        return {"scale_small": self.output_channels["stage_2"], "scale_medium": self.output_channels["stage_3"],
                "scale_large": self.output_channels["stage_4"]}

    def get_stride_factors(self) -> Dict[str, int]:
        return {"scale_small": 8, "scale_medium": 16, "scale_large": 32}
