"""FPN, YOLO head/decoder/loss and the system composition on the HIP path
(reference src/models/feature_fusion.py, yolo_head.py, hybrid_vision.py)."""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .backbone import HybridVisionBackbone
from .layers import ctx_scope, linear_prep, run_conv, to_nchw_view, to_nhwc
from .manifold import ManifoldHyperConnection, prepare_plans
from .runtime import Branches, HVOptions, RunCtx, VersionWatch, current, module_options, require_cuda, use_ctx, PRECISIONS
from .vit import HybridVisionEncoder

# side-stream Sinkhorn + mHC prep (PrepProgram.run overlap) from batch HVOptions.prep_overlap_min_batch
# (8): round 6, base 640 bf16 B=16 graph step 17.30 -> 17.01 / 17.26 -> 17.10 ms (same box, alternating);
# at B=1 (recompute) 5.81 vs 5.85 ms, so off there (profiles/r06/prep_overlap_ab.txt).  Round 1 measured
# it 0.1 ms slower, before the weight prep and the GEMM kernels beside it were rewritten.

# outputs['detections'] keys: the per-scale names DetectionPostprocessor (postprocessing.py:
# 234-244, 270-281) and MHCYOLOLoss (loss_functions.py:86) look up
DETECTION_KEYS = ("small_scale", "medium_scale", "large_scale")

DEFAULT_ANCHORS = [[(10, 13), (16, 30), (33, 23)],
                   [(30, 61), (62, 45), (59, 119)],
                   [(116, 90), (156, 198), (373, 326)]]


def _tokens(mhc: ManifoldHyperConnection, x: torch.Tensor) -> torch.Tensor:
    n, h, w, c = x.shape
    return mhc.forward_tokens(x.view(-1, c)).view(n, h, w, c)


# ====================================================================== FPN
class FeaturePyramidNetwork(nn.Module):
    """feature_fusion.py:10-153 (fusion 'add'; shim S2 on the mHC fusions)."""

    def __init__(self, channels: List[int], use_mhc: bool = True, fusion_method: str = "add",
                 sk_iterations: int = 20):
        super().__init__()
        if fusion_method != "add" or not use_mhc:
            raise NotImplementedError("hv_amd implements the reference default FPN (add, use_mhc)")
        self.channels, self.num_scales, self.fusion_method = channels, len(channels), fusion_method
        self.lateral_convs = nn.ModuleList([nn.Conv2d(c, 256, kernel_size=1) for c in channels])
        self.refinement_convs = nn.ModuleList([nn.Sequential(
            nn.Conv2d(256, 256, 3, padding=1), nn.BatchNorm2d(256), nn.ReLU(inplace=True),
            nn.Conv2d(256, 256, 3, padding=1), nn.BatchNorm2d(256), nn.ReLU(inplace=True))
            for _ in channels])
        self.mhc_fusions = nn.ModuleList([ManifoldHyperConnection(256, expansion_rate=2, sk_iterations=sk_iterations)
                                          for _ in channels])
        self.output_convs = nn.ModuleList([nn.Conv2d(256, oc, kernel_size=1) for oc in [256, 512, 1024][:len(channels)]])
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _refine(self, i: int, x: torch.Tensor) -> torch.Tensor:
        r = self.refinement_convs[i]
        x = run_conv(x, r[0], r[1], "relu", self)
        x = run_conv(x, r[3], r[4], "relu", self)
        return _tokens(self.mhc_fusions[i], x)

    def forward_nhwc(self, feats: Dict[str, torch.Tensor], emit=None) -> Dict[str, torch.Tensor]:
        """emit(key, tensor): called as soon as each fused scale is computed (top-down, large
        first), so a consumer (the detection head on a side stream) can start on it while the
        pyramid continues."""
        pl = run_conv(feats["scale_large"], self.lateral_convs[2], None, "none", self)
        pm = run_conv(feats["scale_medium"], self.lateral_convs[1], None, "none", self)
        ps = run_conv(feats["scale_small"], self.lateral_convs[0], None, "none", self)
        out = {}

        def put(key, t):
            out[key] = t
            if emit is not None:
                emit(key, t)
        rl = self._refine(2, pl)
        put("fused_large", run_conv(rl, self.output_convs[2], None, "none", self))
        rm = self._refine(1, ops.upsample_add(pm, rl))
        put("fused_medium", run_conv(rm, self.output_convs[1], None, "none", self))
        rs = self._refine(0, ops.upsample_add(ps, rm))
        put("fused_small", run_conv(rs, self.output_convs[0], None, "none", self))
        return {k: out[k] for k in ("fused_large", "fused_medium", "fused_small")}

    def forward(self, features: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        if self.training:
            from . import train_model as TM
            from .runtime import resolve_dtype
            dt = resolve_dtype(self.mhc_fusions[0])
            nh = {k: TM.nhwc_in(v, dt) for k, v in features.items() if k.startswith("scale_")}
            return {k: to_nchw_view(v) for k, v in TM.fpn(self, nh, TM.module_H(self)).items()}
        with ctx_scope(self) as ctx:
            nh = {k: to_nhwc(v, ctx.dtype) for k, v in features.items() if k.startswith("scale_")}
            return {k: to_nchw_view(v) for k, v in self.forward_nhwc(nh).items()}


# ====================================================================== YOLO
class YOLOAnchorGenerator(nn.Module):
    """yolo_head.py:11-90 with shim S4: per-scale anchors [S, A, 1, 1, 4] (w, h / 416)."""

    def __init__(self, anchor_sizes=None, grid_sizes: List[int] = (13, 26, 52)):
        super().__init__()
        self.anchor_sizes = anchor_sizes or DEFAULT_ANCHORS
        self.grid_sizes = list(grid_sizes)
        self.num_scales = len(self.grid_sizes)
        self.num_anchors = len(self.anchor_sizes[0])
        rows = [torch.tensor([[0.5, 0.5, w / 416.0, h / 416.0] for (w, h) in s]).view(len(s), 1, 1, 4)
                for s in self.anchor_sizes]
        self.register_buffer("anchors", torch.stack(rows))

    def forward(self, scale_idx: int) -> torch.Tensor:
        return self.anchors[scale_idx]

    def get_num_anchors(self) -> int:
        return self.num_anchors


class YOLOPredictionHead(nn.Module):
    """yolo_head.py:93-203: 3x3 C->2C, 3x3 2C->C (BN, LeakyReLU 0.1), mHC(C), 1x1 -> A*(5+nc)."""

    def __init__(self, in_channels: int, num_classes: int = 80, num_anchors: int = 3, use_mhc: bool = True,
                 sk_iterations: int = 20):
        super().__init__()
        self.in_channels, self.num_classes, self.num_anchors = in_channels, num_classes, num_anchors
        self.output_dim = num_anchors * (5 + num_classes)
        self.conv_layers = nn.Sequential(
            nn.Conv2d(in_channels, in_channels * 2, 3, padding=1), nn.BatchNorm2d(in_channels * 2), nn.LeakyReLU(0.1),
            nn.Conv2d(in_channels * 2, in_channels, 3, padding=1), nn.BatchNorm2d(in_channels), nn.LeakyReLU(0.1))
        self.mhc_enhance = ManifoldHyperConnection(in_channels, expansion_rate=2, sk_iterations=sk_iterations) \
            if use_mhc else nn.Identity()
        self.pred_conv = nn.Conv2d(in_channels, self.output_dim, kernel_size=1)
        for m in self.conv_layers:
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="leaky_relu")
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        nn.init.normal_(self.pred_conv.weight, std=0.01)
        nn.init.zeros_(self.pred_conv.bias)
        with torch.no_grad():
            b = self.pred_conv.bias.view(num_anchors, -1)
            b[:, 4] = -4.0
            b[:, 5:] = -math.log((1 - 0.01) / 0.01) / num_classes

    def logits_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        c = self.conv_layers
        x = run_conv(x, c[0], c[1], "leaky", self)
        x = run_conv(x, c[3], c[4], "leaky", self)
        if isinstance(self.mhc_enhance, ManifoldHyperConnection):
            x = _tokens(self.mhc_enhance, x)
        return run_conv(x, self.pred_conv, None, "none", self)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        require_cuda(x, "YOLOPredictionHead")
        if self.training:
            from . import train_model as TM
            from .runtime import resolve_dtype
            lg = TM.head_logits(self, TM.nhwc_in(x, resolve_dtype(self)), TM.module_H(self))
            n, h, w, _ = lg.shape
            return TM._PredViewFn.apply(lg, self.num_anchors)
        with ctx_scope(self) as ctx:
            lg = self.logits_nhwc(to_nhwc(x, ctx.dtype))
            n, h, w, _ = lg.shape
            return lg.float().view(n, h, w, self.num_anchors, -1).permute(0, 3, 1, 2, 4).contiguous()


class YOLODecoder(nn.Module):
    """yolo_head.py:206-294 with shim S5 (boxes [B, A, H, W, 4], xyxy, normalised)."""

    def __init__(self, image_size: int = 416):
        super().__init__()
        self.image_size = image_size

    def forward(self, predictions: torch.Tensor, anchors: torch.Tensor, grid_size=None) -> Dict[str, torch.Tensor]:
        require_cuda(predictions, "YOLODecoder")
        B, A, H, W, P = predictions.shape
        lg = predictions.float().permute(0, 2, 3, 1, 4).contiguous().view(B, H, W, A * P)
        dec, _ = ops.yolo_decode(lg, A, P - 5, anchors.reshape(A, -1)[:, 2:4].contiguous())
        return dec


class YOLOLoss(nn.Module):
    """yolo_head.py:297-465 on the fused HIP loss kernels (hv_yolo_loss forward + dlogits)."""

    def __init__(self, num_classes: int = 80, anchors=None, image_size: int = 416, lambda_coord: float = 5.0,
                 lambda_noobj: float = 0.5, lambda_obj: float = 1.0, lambda_cls: float = 1.0):
        super().__init__()
        self.num_classes, self.image_size = num_classes, image_size
        self.lambda_coord, self.lambda_noobj, self.lambda_obj, self.lambda_cls = lambda_coord, lambda_noobj, lambda_obj, lambda_cls
        self.anchors = anchors or DEFAULT_ANCHORS
        self.num_scales = len(self.anchors)

    def forward(self, predictions, targets):
        """yolo_head.py:374-465 via the fused loss kernel (hv_yolo_loss): component sums are
        device tensors (no .item() per scale), total_loss is differentiable."""
        from .train_model import yolo_loss_api
        return yolo_loss_api(self, predictions, targets)


class YOLODetectionHead(nn.Module):
    """yolo_head.py:468-756."""

    def __init__(self, in_channels_list: List[int], num_classes: int = 80, anchors=None, use_mhc: bool = True,
                 sk_iterations: int = 20):
        super().__init__()
        self.in_channels_list, self.num_classes, self.num_scales = in_channels_list, num_classes, len(in_channels_list)
        self.anchor_generator = YOLOAnchorGenerator(anchors)
        self.num_anchors = self.anchor_generator.get_num_anchors()
        self.pred_heads = nn.ModuleList([YOLOPredictionHead(c, num_classes, self.num_anchors, use_mhc, sk_iterations)
                                         for c in in_channels_list])
        self.decoder = YOLODecoder(image_size=416)
        self.loss_fn = YOLOLoss(num_classes=num_classes, anchors=anchors)
        self.grid_sizes = [(13, 13), (26, 26), (52, 52)]

    def forward_nhwc(self, feats: Dict[str, torch.Tensor], detections: Optional[Dict[str, torch.Tensor]] = None):
        """detections: if a dict is given, it is filled with the per-scale decoded detections
        tensors (HybridVisionSystem's 'detections' output key)."""
        res = {s: self.scale_nhwc(s, feats[key], detections is not None)
               for s, key in enumerate(("scale_small", "scale_medium", "scale_large")) if key in feats}
        return self.collect(res, detections)

    def scale_nhwc(self, s: int, x: torch.Tensor, want_detections: bool):
        """One scale's prediction head + decode: (pred, decoded dict)."""
        lg = self.pred_heads[s].logits_nhwc(x)
        awh = self.anchor_generator.anchors[s].reshape(self.num_anchors, 4)[:, 2:4].contiguous()
        dec, pred = ops.yolo_decode(lg, self.num_anchors, self.num_classes, awh, detections=want_detections)
        return pred, dec

    @staticmethod
    def collect(res: Dict[int, Tuple], detections: Optional[Dict[str, torch.Tensor]]):
        preds, decoded = {}, {}
        for s in sorted(res):
            pred, dec = res[s]
            if detections is not None:
                detections[DETECTION_KEYS[s]] = dec.pop("detections")
            preds[f"scale_{s}"] = pred
            decoded[f"scale_{s}"] = dec
        return preds, decoded

    def forward(self, features: Dict[str, torch.Tensor], targets=None, compute_loss: bool = False):
        if self.training:
            preds, decoded = {}, {}
            for s, key in enumerate(("scale_small", "scale_medium", "scale_large")):
                if key not in features:
                    continue
                p = self.pred_heads[s](features[key])
                preds[f"scale_{s}"] = p
                decoded[f"scale_{s}"] = self.decoder(p.detach(), self.anchor_generator(s), None)
            out = {"predictions": preds, "decoded": decoded}
            if compute_loss and targets is not None:
                out["loss"] = self.loss_fn(preds, targets)
            return out
        with ctx_scope(self) as ctx:
            nh = {k: to_nhwc(v, ctx.dtype) for k, v in features.items()}
            preds, decoded = self.forward_nhwc(nh)
        out = {"predictions": preds, "decoded": decoded}
        if compute_loss and targets is not None:
            out["loss"] = self.loss_fn(preds, targets)
        return out

    # ---- post-processing (yolo_head.py:571-731) on the GPU: hv_nms, two launches per batch
    def post_process(self, decoded_outputs, confidence_threshold: float = 0.5, iou_threshold: float = 0.5,
                     max_detections: int = 100):
        """Per scale: class_score > threshold, greedy NMS; then NMS across scales.
        One host synchronisation for the whole batch (to cut the per-image lists)."""
        boxes, scores, labels, count = ops.nms_batched(decoded_outputs, confidence_threshold, iou_threshold,
                                                       max_detections)
        out = []
        for b, n in enumerate(count.tolist()):
            if n == 0:
                dev = boxes.device
                out.append({"boxes": torch.tensor([], device=dev), "scores": torch.tensor([], device=dev),
                            "labels": torch.tensor([], device=dev, dtype=torch.long)})
            else:
                out.append({"boxes": boxes[b, :n], "scores": scores[b, :n], "labels": labels[b, :n]})
        return out

    def non_max_suppression(self, boxes, scores, iou_threshold: float = 0.5, max_detections: int = 100):
        if boxes.numel() == 0:
            return torch.tensor([], dtype=torch.long, device=boxes.device)
        order = torch.argsort(scores, descending=True)
        keep = []
        while order.numel() > 0:
            i = order[0]
            keep.append(int(i))
            if len(keep) >= max_detections or order.numel() == 1:
                break
            rest = order[1:]
            order = rest[self.compute_iou(boxes[i].unsqueeze(0), boxes[rest]) < iou_threshold]
        return torch.tensor(keep, dtype=torch.long, device=boxes.device)

    @staticmethod
    def compute_iou(b1, b2):
        ix1 = torch.max(b1[..., 0], b2[..., 0]); iy1 = torch.max(b1[..., 1], b2[..., 1])
        ix2 = torch.min(b1[..., 2], b2[..., 2]); iy2 = torch.min(b1[..., 3], b2[..., 3])
        inter = (ix2 - ix1).clamp(min=0) * (iy2 - iy1).clamp(min=0)
        a1 = (b1[..., 2] - b1[..., 0]) * (b1[..., 3] - b1[..., 1])
        a2 = (b2[..., 2] - b2[..., 0]) * (b2[..., 3] - b2[..., 1])
        return inter / (a1 + a2 - inter + 1e-6)


# ====================================================================== graphs
class GraphRunner:
    """One HybridVisionSystem forward captured as a HIP graph (torch.cuda.CUDAGraph over the
    HIP runtime).  Every kernel of the step -- grouped Sinkhorn, coefficient folds, the token
    path, decode -- is recorded once and replayed with no host launch overhead.

    Staleness: the graph bakes in parameter storage, the storage of the buffers it writes
    (Sinkhorn histories) and, with the model frozen, the prepared coefficients.  Every call
    snapshots the parameters' / buffers' storage pointers and version counters
    (runtime.VersionWatch) BEFORE enqueueing the replay -- a replay after a `.data` swap or a
    buffer rebind would read or write freed storage -- and when anything changed (an optimizer
    step, load_state_dict, a `.data` swap, `.to()`, HVTrainer's flat buffers) it re-captures
    first.  In a replay loop the ~0.4 ms host check still overlaps the previous step on the GPU.

    Ownership: replay() returns the captured static outputs, overwritten by the next replay;
    __call__(x, owned=True) returns fresh copies (one segmented-copy launch)."""

    def __init__(self, model: "HybridVisionSystem", example: torch.Tensor, task: str = "detection"):
        require_cuda(example, "GraphRunner")
        self.model = model
        self.task = task
        self.static_in = example.detach().clone()
        self.recaptures = 0
        self._capture()

    def _capture(self):
        model = self.model
        self.graph = None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):                   # allocate workspaces, upload tables, set attributes
                model(self.static_in, task=self.task)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: other threads (the engine's worker pool) may keep running eager forwards
        # on their own streams while this thread captures
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.static_out, ctx = model.forward_eval(self.static_in, task=self.task)
        # the graph reads buffers that live outside its memory pool (the grouped Sinkhorn /
        # coefficient-prep program and its device tables, frozen plans): keep THIS capture's
        # RunCtx alive (the one its forward returned -- not a per-model "latest" slot another
        # thread's forward may have overwritten), or a later set_options / set_precision / cache
        # rebuild would free them under it
        self.ctx = ctx
        self.version = model._watch.snapshot()

    def replay(self) -> Dict[str, Any]:
        if self.model._watch.snapshot() != self.version:
            self.recaptures += 1
            self._capture()
        self.graph.replay()
        return self.static_out

    def __call__(self, x: torch.Tensor, owned: bool = False) -> Dict[str, Any]:
        self.static_in.copy_(x)
        out = self.replay()
        return ops.clone_tree(out) if owned else out


# ====================================================================== system
class HybridVisionSystem(nn.Module):
    """hybrid_vision.py:17-485.  Accepts the real constructor ``(config)`` and the call-site
    form ``(config=..., num_classes=..., use_vit=..., use_rag=...)`` of scripts/train.py:189-194
    (SURVEY §8b).  Extra build knobs: num_blocks, vit_depth, sk_iters, precision ('bf16'|'fp32').
    """

    def __init__(self, config: Optional[Dict[str, Any]] = None, **kwargs):
        super().__init__()
        cfg = dict(config or {})
        cfg.update(kwargs)
        self.config = cfg
        self.image_size = cfg.get("image_size", 416)
        self.num_classes = cfg.get("num_classes", 80)
        self.use_mhc = cfg.get("use_mhc", True)
        self.use_vit = cfg.get("use_vit", True)
        self.use_rag = cfg.get("use_rag", False)
        self.use_fpn = cfg.get("use_fpn", True)
        self.has_segmentation = cfg.get("has_segmentation", False)
        self.has_depth = cfg.get("has_depth", False)
        if self.use_rag or not self.use_fpn or not self.use_mhc or self.has_segmentation or self.has_depth:
            raise NotImplementedError("hv_amd builds the reference default system (use_mhc, use_fpn; RAG, "
                                      "segmentation and depth heads are out of scope, SURVEY §2)")
        it = int(cfg.get("sk_iters", 20))
        self.hv_precision = cfg.get("precision", "bf16")
        self.backbone = HybridVisionBackbone(3, 32, list(cfg.get("num_blocks", [2, 3, 4, 2])), True, "silu", 0.1,
                                             sk_iterations=it, verbose=cfg.get("verbose", True))
        bc = self.backbone.get_output_channels()
        if self.use_vit:
            self.vit_encoder = HybridVisionEncoder(bc["scale_large"], 256, int(cfg.get("vit_depth", 6)), 8, True,
                                                   sk_iterations=it)
        self.feature_fusion = FeaturePyramidNetwork([bc["scale_small"], bc["scale_medium"], bc["scale_large"]],
                                                    True, "add", sk_iterations=it)
        fused = [256, 512, 1024]
        self.detection_head = YOLODetectionHead(fused, self.num_classes, cfg.get("anchors"), True, sk_iterations=it)
        self.final_fusion = ManifoldHyperConnection(sum(fused), expansion_rate=2, sk_iterations=it)
        self.output_projection = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(sum(fused), 512),
                                               nn.ReLU(), nn.Linear(512, 256))
        for m in self.modules():                              # hybrid_vision.py:183-197
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        self._mhc_modules = [m for m in self.modules() if isinstance(m, ManifoldHyperConnection)]
        from .manifold import MultiHeadManifoldAttention
        self._qkv_groups = {id(a): (a.q_proj, a.k_proj, a.v_proj) for a in self.modules()
                            if isinstance(a, MultiHeadManifoldAttention)}
        self._frozen: Optional[Tuple[Any, RunCtx]] = None
        self._sk_cache: Dict[str, Any] = {}
        self._watch = VersionWatch(self)

    # ---- precision / caching controls
    def set_precision(self, precision: str) -> "HybridVisionSystem":
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {list(PRECISIONS)}")
        self.hv_precision = precision
        self._frozen = None
        return self

    def set_options(self, options: Optional[HVOptions] = None, **kw) -> "HybridVisionSystem":
        """Per-model execution options (runtime.HVOptions: kernel variants, exact restructurings);
        e.g. ``model.set_options(use_fused_mhc=False)``.  Prepared / frozen state is rebuilt; a
        captured GraphRunner keeps the options it was captured with."""
        base = options if options is not None else module_options(self)
        self.hv_options = base.replace(**kw) if kw else base
        self._frozen = None if self._frozen is None else (None, None)
        self._sk_cache = {}
        return self

    def freeze(self, enabled: bool = True) -> "HybridVisionSystem":
        """Eval/streaming: keep the prepared coefficients (Sinkhorn, folds, BN folds, casts)
        across forwards until any parameter changes (version counters are checked)."""
        self._frozen = (None, None) if enabled else None
        return self

    def _make_ctx(self, batch: int = 1) -> RunCtx:
        opts = module_options(self)
        ctx = RunCtx(dtype=PRECISIONS[self.hv_precision], opts=opts)
        key = tuple(t.data_ptr() for t in self.parameters()) + tuple(t.data_ptr() for t in self.buffers())
        overlap = opts.prep_overlap or batch >= opts.prep_overlap_min_batch
        prepare_plans(self._mhc_modules, ctx, self._sk_cache, key, overlap=overlap, groups=self._qkv_groups)
        return ctx

    def capture(self, example: torch.Tensor, task: str = "detection") -> "GraphRunner":
        """Capture one full forward (coefficient prep included unless frozen) into a HIP
        graph; the returned runner copies its input into the captured buffer and replays."""
        return GraphRunner(self, example, task)

    def _ctx(self, batch: int = 1) -> RunCtx:
        if self._frozen is None:
            return self._make_ctx(batch)
        ver = self._watch.snapshot()
        if self._frozen[0] != ver:
            self._frozen = (ver, self._make_ctx(batch))
        return self._frozen[1]

    # ---- forward (hybrid_vision.py:222-367)
    def forward(self, x: torch.Tensor, targets=None, text_query=None, task: str = "detection",
                compute_loss: bool = False) -> Dict[str, Any]:
        require_cuda(x, "HybridVisionSystem")
        if self.training:
            # training step: BN batch statistics, dropout, autograd over HIP kernels
            from .train_model import system_forward
            return system_forward(self, x, targets, task, compute_loss)
        return self.forward_eval(x, targets, task, compute_loss)[0]

    def forward_eval(self, x: torch.Tensor, targets=None, task: str = "detection",
                     compute_loss: bool = False) -> Tuple[Dict[str, Any], RunCtx]:
        """The eval forward, returning also the RunCtx it ran under (the prepared coefficients and
        device tables its kernels read): a graph capture pins exactly that context.  Re-entrant --
        nothing per call is stored on the module, so concurrent forwards from several threads
        (the engine's worker pool) do not interfere."""
        require_cuda(x, "HybridVisionSystem")
        ctx = self._ctx(x.shape[0])
        with torch.no_grad(), use_ctx(ctx):
            # independent parts on side streams (runtime.Branches): base 640 bf16 B=16 graph step
            # 17.37 vs 17.85 ms; at B=1 the cross-stream edges cost more than the overlap wins
            # (frozen p50 4.61 vs 4.46 ms; profiles/r05/branches_ab.txt)
            br = Branches(x.shape[0] >= ctx.opts.branch_min_batch)
            if x.dtype == torch.float32 and x.is_contiguous():
                bb = self.backbone.forward_nhwc(None, image=x, branches=br)   # direct stem conv from NCHW
            else:
                bb = self.backbone.forward_nhwc(to_nhwc(x, ctx.dtype), branches=br)
            outputs: Dict[str, Any] = {}
            if self.use_vit:
                vit = self.vit_encoder.forward_nhwc(bb["scale_large"])
                bb["scale_large"] = ops.add_scaled(bb["scale_large"], vit, 0.5)
                outputs["vit_features"] = to_nchw_view(vit)
            head_res: Dict[int, Tuple] = {}
            emit = None
            if task == "detection":
                # each scale's head starts on a side stream as soon as the pyramid has produced it
                scale_of = {"fused_small": 0, "fused_medium": 1, "fused_large": 2}

                def emit(key, t):
                    s = scale_of[key]
                    head_res[s] = br.fork(lambda: self.detection_head.scale_nhwc(s, t, True))
            fused = self.feature_fusion.forward_nhwc(bb, emit)
            if task == "detection":
                dets: Dict[str, torch.Tensor] = {}
                preds, decoded = self.detection_head.collect(head_res, dets)
                outputs["predictions"] = preds
                outputs["decoded"] = decoded
                outputs["detections"] = dets
                if compute_loss and targets is not None:
                    br.join()
                    outputs["loss"] = self.detection_head.loss_fn(preds, targets)
            final = self._final_features(fused)
            if task == "features":
                outputs["all_features"] = {"backbone": {k: to_nchw_view(v) for k, v in bb.items() if k != "raw_features"},
                                           "fused": {k: to_nchw_view(v) for k, v in fused.items()}, "final": final}
            bbv = {k: to_nchw_view(v) for k, v in bb.items() if k != "raw_features"}
            bbv["raw_features"] = {k: to_nchw_view(v) for k, v in bb["raw_features"].items()}
            outputs["backbone_features"] = bbv
            outputs["fused_features"] = {k: to_nchw_view(v) for k, v in fused.items()}
            outputs["final_features"] = final
            br.join()                          # every branch's results are on the forward's stream
        ctx.join_prep()                        # side-stream prep joined even if no mHC ran
        return outputs, ctx

    def _final_features(self, fused: Dict[str, torch.Tensor]) -> torch.Tensor:
        """hybrid_vision.py:369-402 with shim S6: GAP x3 -> cat -> mHC(1792) -> Linear/ReLU/Linear."""
        pooled = torch.cat([ops.channel_mean(fused[k]) for k in ("fused_small", "fused_medium", "fused_large")], 1)
        dt = current().dtype
        c = self.final_fusion.forward_tokens(pooled.to(dt).contiguous())
        w2, b2 = linear_prep(self.output_projection[2], dt)
        w4, b4 = linear_prep(self.output_projection[4], dt)
        h = ops.gemm(c, w2, bias=b2, act="relu")
        return ops.gemm(h, w4, bias=b4, out_dtype=torch.float32)

    def detect(self, x, confidence_threshold: float = 0.5, iou_threshold: float = 0.5, max_detections: int = 100,
               text_query=None):
        out = self.forward(x, text_query=text_query, task="detection")
        return self.detection_head.post_process(out["decoded"], confidence_threshold, iou_threshold, max_detections)

    def get_stability_metrics(self) -> Dict[str, Any]:
        """hybrid_vision.py:441-457 with shim S7 (root module skipped)."""
        metrics = {}
        for name, m in self.named_modules():
            if m is self or not hasattr(m, "get_stability_metrics"):
                continue
            for k, v in m.get_stability_metrics().items():
                metrics[f"{name}.{k}"] = v
        return metrics

    def get_parameter_count(self) -> Dict[str, int]:
        counts = {name: sum(p.numel() for p in m.parameters()) for name, m in self.named_children()}
        counts["total"] = sum(p.numel() for p in self.parameters())
        counts["trainable"] = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return counts
