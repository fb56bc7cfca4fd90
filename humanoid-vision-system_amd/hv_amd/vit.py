"""mHC transformer encoder on the HIP path (reference src/models/vit_encoder_decoder.py)."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .layers import conv_prep, ctx_scope, linear_prep, run_conv, to_nchw_view, to_nhwc
from .manifold import ManifoldHyperConnection, MultiHeadManifoldAttention, RMSNorm
from .runtime import current, options, require_cuda


def _positions(pe: torch.Tensor, tokens: int) -> torch.Tensor:
    """[1, L+1, D] learned table -> [tokens+1, D]; shim S3: interpolate the L patch slots."""
    ctx = current()
    key = ("pos", id(pe), tokens)
    if ctx is not None and key in ctx.plans:
        return ctx.plans[key]
    t = ops.f32(pe[0])
    if t.shape[0] != tokens + 1:
        t = torch.cat([t[:1], ops.interp_linear(t[1:], tokens)], dim=0)
    if ctx is not None:
        ctx.plans[key] = t
    return t


# HVOptions.cls_only_last_block: run the encoder's last block on the CLS rows only
# (TransformerEncoderBlock.forward_tokens_cls)


class PatchEmbedding(nn.Module):
    """vit_encoder_decoder.py:11-108 (patch_size 1 use: 1x1 projection over the CNN grid)."""

    def __init__(self, image_size: int = 224, patch_size: int = 16, in_channels: int = 3,
                 embed_dim: int = 768, use_mhc: bool = True, sk_iterations: int = 20):
        super().__init__()
        if not use_mhc:
            raise NotImplementedError("hv_amd implements use_mhc=True (reference default)")
        self.image_size, self.patch_size, self.in_channels, self.embed_dim = image_size, patch_size, in_channels, embed_dim
        self.num_patches = (image_size // patch_size) ** 2
        self.projection = nn.Conv2d(in_channels, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.mhc_enhance = ManifoldHyperConnection(embed_dim, expansion_rate=2, sk_iterations=sk_iterations)
        self.position_embeddings = nn.Parameter(torch.zeros(1, self.num_patches + 1, embed_dim))
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.norm = RMSNorm(embed_dim)
        nn.init.trunc_normal_(self.position_embeddings, std=0.02)
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        nn.init.xavier_uniform_(self.projection.weight)
        nn.init.zeros_(self.projection.bias)

    def forward_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        """x NHWC [n, h, w, C] -> tokens [n, h*w+1, D]."""
        t = run_conv(x, self.projection, None, "none", self)
        n, h, w, d = t.shape
        t = self.mhc_enhance.forward_tokens(t.view(-1, d))
        pos = _positions(self.position_embeddings, h * w)
        return ops.vit_tokens(t.view(n, h * w, d), self.cls_token.view(-1), pos, self.norm.scale)

    def forward(self, x):
        require_cuda(x, "PatchEmbedding")
        with ctx_scope(self) as ctx:
            return self.forward_nhwc(to_nhwc(x, ctx.dtype))


class TransformerEncoderBlock(nn.Module):
    """vit_encoder_decoder.py:111-210 (pre-RMSNorm, mHC attention, MLP, mHC residuals)."""

    def __init__(self, embed_dim: int = 768, num_heads: int = 8, mlp_ratio: float = 4.0, dropout: float = 0.1,
                 use_mhc: bool = True, sk_iterations: int = 20):
        super().__init__()
        if not use_mhc:
            raise NotImplementedError("hv_amd implements use_mhc=True (reference default)")
        self.embed_dim, self.num_heads, self.use_mhc = embed_dim, num_heads, use_mhc
        self.attention = MultiHeadManifoldAttention(embed_dim, num_heads, dropout, use_mhc,
                                                    sk_iterations=sk_iterations)
        self.norm1 = RMSNorm(embed_dim)
        hid = int(embed_dim * mlp_ratio)
        self.mlp = nn.Sequential(nn.Linear(embed_dim, hid), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hid, embed_dim), nn.Dropout(dropout))
        self.norm2 = RMSNorm(embed_dim)
        self.residual_mhc1 = ManifoldHyperConnection(embed_dim, expansion_rate=2, sk_iterations=sk_iterations)
        self.residual_mhc2 = ManifoldHyperConnection(embed_dim, expansion_rate=2, sk_iterations=sk_iterations)
        self.dropout = nn.Dropout(dropout)

    def forward_tokens(self, x: torch.Tensor, n: int) -> torch.Tensor:
        """x: [n*L, D] residual stream (compute dtype)."""
        h = ops.rmsnorm(x, ops.f32(self.norm1.scale))
        a = self.attention.forward_tokens(h, n)
        x = self.residual_mhc1.forward_tokens(a, residual=x)
        h = ops.rmsnorm(x, ops.f32(self.norm2.scale))
        w0, b0 = linear_prep(self.mlp[0], x.dtype)
        w3, b3 = linear_prep(self.mlp[3], x.dtype)
        h = ops.gemm(ops.gemm(h, w0, bias=b0, act="gelu"), w3, bias=b3)
        return self.residual_mhc2.forward_tokens(h, residual=x)

    def forward_tokens_cls(self, x: torch.Tensor, n: int) -> torch.Tensor:
        """The block's output rows for the CLS tokens only, [n, D] (x: [n*L, D]).  Exact for a
        final block whose only consumer is the CLS token (VisionTransformerEncoder :308-311,
        HybridVisionEncoder :505-511): every op after attention's key/value projections is
        per-token, so q_proj, out_proj, residual_mhc1, the MLP and residual_mhc2 run on n rows
        instead of n*L (k_proj / v_proj still see every token)."""
        L = x.shape[0] // n
        att = self.attention
        h = ops.rmsnorm(x, ops.f32(self.norm1.scale))
        h_cls = ops.gather_rows(h, L)
        x_cls = ops.gather_rows(x, L)
        q = att.q_proj.forward_tokens(h_cls).view(n, 1, -1)
        k = att.k_proj.forward_tokens(h).view(n, L, -1)
        v = att.v_proj.forward_tokens(h).view(n, L, -1)
        o, _ = ops.attention_general(q, k, v, att.num_heads)
        a = att.out_proj.forward_tokens(o.view(n, -1))
        x_cls = self.residual_mhc1.forward_tokens(a, residual=x_cls)
        h = ops.rmsnorm(x_cls, ops.f32(self.norm2.scale))
        w0, b0 = linear_prep(self.mlp[0], x.dtype)
        w3, b3 = linear_prep(self.mlp[3], x.dtype)
        h = ops.gemm(ops.gemm(h, w0, bias=b0, act="gelu"), w3, bias=b3)
        return self.residual_mhc2.forward_tokens(h, residual=x_cls)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        require_cuda(x, "TransformerEncoderBlock")
        if self.training:
            from . import train_model as TM
            from .runtime import resolve_dtype
            n, L, D = x.shape
            t = x.reshape(n * L, D).float().contiguous()        # the block's residual stream is fp32
            return TM.encoder_block(self, t, n, TM.module_H(self),
                                    resolve_dtype(self.residual_mhc1)).view(n, L, D).to(x.dtype)
        with ctx_scope(self) as ctx:
            n, L, D = x.shape
            t = x.reshape(n * L, D).to(ctx.dtype).contiguous()
            return self.forward_tokens(t, n).view(n, L, D).to(x.dtype)


class VisionTransformerEncoder(nn.Module):
    """vit_encoder_decoder.py:213-333 (num_classes=0: returns the normalised CLS token)."""

    def __init__(self, image_size: int = 224, patch_size: int = 16, in_channels: int = 3, embed_dim: int = 768,
                 depth: int = 12, num_heads: int = 12, mlp_ratio: float = 4.0, dropout: float = 0.1,
                 use_mhc: bool = True, num_classes: int = 1000, sk_iterations: int = 20):
        super().__init__()
        self.image_size, self.patch_size, self.embed_dim, self.depth, self.use_mhc = \
            image_size, patch_size, embed_dim, depth, use_mhc
        if patch_size != 1:
            raise NotImplementedError("hv_amd runs the patch_size=1 encoder of HybridVisionEncoder")
        self.patch_embed = PatchEmbedding(image_size, patch_size, in_channels, embed_dim, use_mhc, sk_iterations)
        self.blocks = nn.ModuleList([TransformerEncoderBlock(embed_dim, num_heads, mlp_ratio, dropout, use_mhc,
                                                             sk_iterations) for _ in range(depth)])
        self.norm = RMSNorm(embed_dim)
        self.head = nn.Linear(embed_dim, num_classes) if num_classes > 0 else nn.Identity()

    def forward_nhwc(self, x: torch.Tensor, features=None, head: bool = True) -> torch.Tensor:
        """x NHWC -> CLS [n, D] (through the head if `head`); `features` (a list) receives the
        token tensors [n, L, D] after the patch embedding and after every block."""
        t = self.patch_embed.forward_nhwc(x)                 # [n, L, D]
        n, L, D = t.shape
        if features is not None:
            features.append(t)
        t = t.view(n * L, D)
        nb = len(self.blocks)
        for i, blk in enumerate(self.blocks):
            if i == nb - 1 and features is None and options().cls_only_last_block:
                cls = blk.forward_tokens_cls(t, n)          # only the CLS rows survive (exact)
                break
            t = blk.forward_tokens(t, n)
            if features is not None:
                features.append(t.view(n, L, D))
        else:
            cls = ops.gather_rows(t, L)
        cls = ops.rmsnorm(cls, ops.f32(self.norm.scale))
        if head and isinstance(self.head, nn.Linear):
            w, b = linear_prep(self.head, cls.dtype)
            cls = ops.gemm(cls, w, bias=b)
        return cls

    def forward(self, x: torch.Tensor, return_features: bool = False):
        """vit_encoder_decoder.py:277-315: output, or (output, [patch tokens, block outputs...])."""
        require_cuda(x, "VisionTransformerEncoder")
        feats = [] if return_features else None
        if self.training:
            from . import train_model as TM
            from .runtime import resolve_dtype
            out = TM.vit_encoder(self, TM.nhwc_in(x, resolve_dtype(self.patch_embed.mhc_enhance)), TM.module_H(self),
                                 features=feats)
        else:
            with ctx_scope(self) as ctx:
                out = self.forward_nhwc(to_nhwc(x, ctx.dtype), feats)
        return (out, feats) if return_features else out

    def extract_features(self, x: torch.Tensor) -> torch.Tensor:
        """vit_encoder_decoder.py:317-333: the normalised CLS token, without the head."""
        require_cuda(x, "VisionTransformerEncoder")
        if self.training:
            from . import train_model as TM
            from .runtime import resolve_dtype
            return TM.vit_encoder(self, TM.nhwc_in(x, resolve_dtype(self.patch_embed.mhc_enhance)), TM.module_H(self),
                                  head=False)
        with ctx_scope(self) as ctx:
            return self.forward_nhwc(to_nhwc(x, ctx.dtype), head=False)


class HybridVisionEncoder(nn.Module):
    """vit_encoder_decoder.py:409-520 with shims S2 (fusion mHC channels-last) and S3."""

    def __init__(self, cnn_channels: int = 512, vit_embed_dim: int = 256, vit_depth: int = 6,
                 vit_num_heads: int = 8, use_mhc: bool = True, sk_iterations: int = 20):
        super().__init__()
        self.cnn_to_vit = nn.Conv2d(cnn_channels, vit_embed_dim, kernel_size=1)
        self.pos_embed = nn.Parameter(torch.zeros(1, 256, vit_embed_dim))
        self.vit_encoder = VisionTransformerEncoder(image_size=16, patch_size=1, in_channels=vit_embed_dim,
                                                    embed_dim=vit_embed_dim, depth=vit_depth,
                                                    num_heads=vit_num_heads, mlp_ratio=4.0, dropout=0.1,
                                                    use_mhc=use_mhc, num_classes=0, sk_iterations=sk_iterations)
        self.vit_to_cnn = nn.Conv2d(vit_embed_dim, cnn_channels, kernel_size=1)
        self.fusion_mhc = ManifoldHyperConnection(cnn_channels, expansion_rate=2, sk_iterations=sk_iterations)
        nn.init.trunc_normal_(self.pos_embed, std=0.02)

    def forward_nhwc(self, cnn: torch.Tensor) -> torch.Tensor:
        n, h, w, c = cnn.shape
        ctx = current()
        key = ("pos_outer", id(self), h * w)
        pos = ctx.plans.get(key) if ctx is not None else None
        if pos is None:
            pe = ops.f32(self.pos_embed[0])
            pos = pe if pe.shape[0] == h * w else ops.interp_linear(pe, h * w)
            if ctx is not None:
                ctx.plans[key] = pos
        # 1x1 conv + bias + positional table (broadcast over images) in one GEMM epilogue
        wv, _, bv = conv_prep(self.cnn_to_vit, None, cnn.dtype, self)
        v = ops.gemm(cnn.view(-1, c), wv, bias=bv, residual=pos, residual_mod=h * w).view(n, h, w, -1)
        cls = self.vit_encoder.forward_nhwc(v)                              # [n, D]
        wt, _, bt = conv_prep(self.vit_to_cnn, None, cnn.dtype, self)
        e = ops.gemm(cls, wt, bias=bt, out_dtype=torch.float32)            # 1x1 conv of the broadcast CLS
        fused = ops.add_rowvec(cnn, e)
        return self.fusion_mhc.forward_tokens(fused.view(-1, c)).view(n, h, w, c)

    def forward(self, cnn_features: torch.Tensor) -> torch.Tensor:
        require_cuda(cnn_features, "HybridVisionEncoder")
        if self.training:
            from . import train_model as TM
            from .runtime import resolve_dtype
            x = TM.nhwc_in(cnn_features, resolve_dtype(self.fusion_mhc))
            return to_nchw_view(TM.hybrid_encoder(self, x, TM.module_H(self)))
        with ctx_scope(self) as ctx:
            return to_nchw_view(self.forward_nhwc(to_nhwc(cnn_features, ctx.dtype)))
