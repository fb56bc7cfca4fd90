"""Synthetic COCO-like detection targets in the reference's YOLOLoss format (SURVEY §8d config C,
§8f-3).  The reference has no grid-assignment code (its dataset returns padded boxes,
data/dataset.py:249-294); YOLOLoss (yolo_head.py:374-465) consumes per-scale grids
[B, A, H, W, 5+C] and regresses the RAW box logits against target[..., :4].  This builder
fills them the way the decoder inverts (yolo_head.py:240-262): for the anchor with the best
w/h IoU, t_xy = logit(offset of the centre inside its cell), t_wh = log(box_wh / anchor_wh),
objectness 1, one-hot class.

Host-side (numpy) data generation; the result is copied to the device once per batch.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

DEFAULT_ANCHORS = [[(10, 13), (16, 30), (33, 23)],
                   [(30, 61), (62, 45), (59, 119)],
                   [(116, 90), (156, 198), (373, 326)]]


def synthetic_boxes(batch: int, seed: int, mean_boxes: float = 7.3, num_classes: int = 80):
    """Per image K ~ Poisson(7.3) boxes: cx, cy ~ U(0,1), w, h ~ logU(0.02, 0.6), label ~ U{0..79}."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(batch):
        k = max(1, int(rng.poisson(mean_boxes)))
        cxcy = rng.uniform(0.0, 1.0, size=(k, 2))
        wh = np.exp(rng.uniform(np.log(0.02), np.log(0.6), size=(k, 2)))
        lab = rng.integers(0, num_classes, size=k)
        out.append((np.concatenate([cxcy, wh], 1).astype(np.float32), lab.astype(np.int64)))
    return out


def assign(boxes, image_size: int, grids: Sequence[Tuple[int, int]], anchors=None, num_classes: int = 80,
           anchor_norm: float = 416.0) -> List[torch.Tensor]:
    """Boxes (normalised cxcywh + labels, per image) -> per-scale target grids [B, A, H, W, 5+C]."""
    anchors = anchors or DEFAULT_ANCHORS
    A = len(anchors[0])
    P = 5 + num_classes
    B = len(boxes)
    tg = [np.zeros((B, A, h, w, P), dtype=np.float32) for (h, w) in grids]
    flat = [(s, a, aw / anchor_norm, ah / anchor_norm) for s in range(len(anchors))
            for a, (aw, ah) in enumerate(anchors[s])]
    for b, (bx, lab) in enumerate(boxes):
        for (cx, cy, w, h), c in zip(bx, lab):
            best, bi = -1.0, 0
            for i, (_, _, aw, ah) in enumerate(flat):
                inter = min(w, aw) * min(h, ah)
                iou = inter / (w * h + aw * ah - inter)
                if iou > best:
                    best, bi = iou, i
            s, a, aw, ah = flat[bi]
            gh, gw = grids[s]
            gx, gy = min(int(cx * gw), gw - 1), min(int(cy * gh), gh - 1)
            ox = np.clip(cx * gw - gx, 0.01, 0.99)
            oy = np.clip(cy * gh - gy, 0.01, 0.99)
            t = tg[s][b, a, gy, gx]
            t[0] = np.log(ox / (1 - ox))
            t[1] = np.log(oy / (1 - oy))
            t[2] = np.log(w / aw)
            t[3] = np.log(h / ah)
            t[4] = 1.0
            t[5:] = 0.0
            t[5 + c] = 1.0
    return [torch.from_numpy(t) for t in tg]


def synthetic_targets(batch: int, image_size: int, seed: int, num_classes: int = 80, strides=(8, 16, 32),
                      anchors=None) -> List[torch.Tensor]:
    grids = [(image_size // s, image_size // s) for s in strides]
    return assign(synthetic_boxes(batch, seed, num_classes=num_classes), image_size, grids, anchors, num_classes)
