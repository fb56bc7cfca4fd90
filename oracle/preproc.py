"""CPU restatement of the reference's default image preprocessing resize (parity ORACLE).

TEST INFRASTRUCTURE ONLY (see oracle/hv_oracle.py header for the usage rule).

The reference (src/inference/preprocessing.py:181-276, PreprocessingMode.FAST without kornia --
kornia is not in requirements.txt) converts BGR->RGB (:202-205) and runs torchvision
``Resize((h, w))`` on a PIL image (:104-110, :268-274), i.e. Pillow ``Image.resize(BILINEAR)``
(Pillow==10.0.0, requirements.txt:6).  The algorithm lives in Pillow's libImaging/Resample.c
(precompute_coeffs, normalize_coeffs_8bpc, ImagingResampleHorizontal_8bpc / Vertical_8bpc):
a triangle filter whose support scales with the downscale factor, coefficients rounded to
22-bit fixed point, a uint8-rounded horizontal pass then a uint8-rounded vertical pass.  This
module restates it in numpy integer arithmetic; it is pinned bit-for-bit by
tests/golden/preproc_pil_* (made by Pillow itself, oracle/gen_golden.py G7).
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def coeffs(in_size: int, out_size: int):
    """precompute_coeffs (bilinear, support 1.0) + normalize_coeffs_8bpc -> (bounds [out, 2], kk [out, ksize])."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum(w)
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else int(0.5 + k * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(v: np.ndarray) -> np.ndarray:
    return np.clip(v >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bilinear_pil(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """uint8 [h, w, 3] -> uint8 [out_h, out_w, 3], Pillow-exact."""
    h, w, _ = img.shape
    hb, hk = coeffs(w, out_w)
    vb, vk = coeffs(h, out_h)
    src = img.astype(np.int64)
    tmp = np.empty((h, out_w, 3), dtype=np.uint8)
    for xx in range(out_w):
        xmin, xn = hb[xx]
        acc = np.full((h, 3), 1 << (PRECISION_BITS - 1), dtype=np.int64)
        acc += np.einsum("hkc,k->hc", src[:, xmin:xmin + xn, :], hk[xx, :xn])
        tmp[:, xx] = _clip8(acc)
    t = tmp.astype(np.int64)
    out = np.empty((out_h, out_w, 3), dtype=np.uint8)
    for yy in range(out_h):
        ymin, yn = vb[yy]
        acc = np.full((out_w, 3), 1 << (PRECISION_BITS - 1), dtype=np.int64)
        acc += np.einsum("kwc,k->wc", t[ymin:ymin + yn], vk[yy, :yn])
        out[yy] = _clip8(acc)
    return out


def preprocess_frames(bgr: np.ndarray, out_h: int, out_w: int,
                      mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """uint8 BGR [n, h, w, 3] -> (resized RGB uint8 [n, out_h, out_w, 3], fp32 NCHW tensor as
    torchvision ToTensor + Normalize computes it: (u / 255 - mean) / std)."""
    import torch
    rgb = np.stack([resize_bilinear_pil(f[:, :, ::-1], out_h, out_w) for f in bgr])
    t = torch.from_numpy(rgb).permute(0, 3, 1, 2).float().div(255)
    t = (t - torch.tensor(mean).view(1, 3, 1, 1)) / torch.tensor(std).view(1, 3, 1, 1)
    return rgb, t
