"""Inference engine with the reference API (src/inference/engine.py:33-671), MI355X edition.

Same public surface -- InferenceConfig fields, InferenceEngine(config, model=None) (and the
call-site form InferenceEngine(model=..., config=..., device=...) of scripts/inference.py:427),
infer / inference / infer_batch / async_infer / get_performance_stats / get_stability_report /
reset_stats, AsyncInferenceEngine.infer_async / infer_sync -- with these differences:
  * the model forward runs on the HIP kernels of hv_amd (bf16 activations, fp32
    coefficients) instead of torch.cuda.amp fp16 autocast; use_half_precision selects bf16;
  * streaming (batch 1) can replay a hipGraph of the whole forward with the coefficients
    frozen (config.use_graphs); the replay is re-captured when any parameter changes and
    infer() returns owned copies of its outputs (GraphRunner);
  * every infer() result carries 'stability_metrics' like the reference, as a lazy mapping:
    the 76 modules' host reads happen on first access, not per frame (collect_stability=True
    also materialises and records them for get_stability_report);
  * forward outputs also carry 'detections' (post-processed boxes / scores / labels per
    image), the key scripts/inference.py:121 reads;
  * the reference preprocessor's stale-cache defect is not reproduced.
"""
from __future__ import annotations

import asyncio
import logging
import queue
import threading
import time
from collections import deque
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from collections.abc import Mapping
from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np
import torch
import torch.nn.functional as F  # noqa: F401

from . import ops
from .runtime import PRECISIONS as PRECISION_DTYPES

logger = logging.getLogger(__name__)

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


@dataclass
class InferenceConfig:
    """engine.py:33-63 (+ use_graphs / collect_stability)."""
    device: str = "cuda"
    use_half_precision: bool = True
    use_tensorrt: bool = False
    tensorrt_precision: str = "FP16"
    batch_size: int = 1
    max_batch_size: int = 16
    warmup_iterations: int = 10
    enable_batching: bool = True
    model_path: str = ""
    input_height: int = 416
    input_width: int = 416
    num_classes: int = 80
    confidence_threshold: float = 0.25
    iou_threshold: float = 0.45
    enable_profiling: bool = False
    log_interval: int = 100
    memory_monitoring: bool = True
    max_latency_ms: int = 50
    target_fps: int = 30
    use_graphs: bool = False
    collect_stability: bool = False
    # frame resize: 'pil' = the reference's default (torchvision Resize on PIL, Pillow-exact),
    # 'bilinear' = its kornia path (F.interpolate bilinear, align_corners=False)
    resample: str = "pil"


def preprocess_image(img: np.ndarray, height: int, width: int, device, dtype=torch.float32,
                     resample: str = "pil") -> torch.Tensor:
    """uint8 HWC BGR frame -> normalised CHW (preprocessing.py:181-276 semantics: BGR->RGB,
    resize, /255, ImageNet mean/std) in one HIP launch (hv_preprocess_pil / hv_preprocess)."""
    return preprocess_frames([img], height, width, device, dtype, resample)[0]


def preprocess_frames(imgs: List[np.ndarray], height: int, width: int, device, dtype=torch.float32,
                      resample: str = "pil") -> torch.Tensor:
    """Batch of same-size uint8 HWC BGR frames -> [n, 3, height, width]: one host->device copy
    of the raw bytes, one preprocessing launch."""
    if imgs[0].dtype != np.uint8 or imgs[0].ndim != 3 or imgs[0].shape[2] != 3:
        raise ValueError("expected uint8 HWC 3-channel frames")
    raw = torch.from_numpy(np.ascontiguousarray(np.stack(imgs))).to(device, non_blocking=True)
    return ops.preprocess(raw, height, width, bgr=True, dtype=dtype, resample=resample)


class LazyStabilityMetrics(Mapping):
    """model.get_stability_metrics() (hybrid_vision.py:441-457), evaluated on first access:
    the reference syncs the host ~300 times per frame for it (engine.py:300-302); streaming
    callers that never read it pay nothing."""

    def __init__(self, model):
        self._model = model
        self._data: Optional[Dict[str, Any]] = None

    def _get(self) -> Dict[str, Any]:
        if self._data is None:
            self._data = self._model.get_stability_metrics() if hasattr(self._model, "get_stability_metrics") else {}
        return self._data

    def __getitem__(self, k):
        return self._get()[k]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())


class InferenceEngine:
    """engine.py:72-562."""

    def __init__(self, config: Optional[InferenceConfig] = None, model: Optional[torch.nn.Module] = None,
                 device: Optional[str] = None, **kw):
        if config is None:
            config = InferenceConfig()
        elif isinstance(config, dict):
            config = InferenceConfig(**{k: v for k, v in config.items() if k in InferenceConfig.__dataclass_fields__})
        if device is not None:
            config.device = str(device)
        self.config = config
        self.device = torch.device(config.device)
        self.use_half = config.use_half_precision and self.device.type == "cuda"
        self.model = model
        if model is None and config.model_path:
            self._load_model()
        elif model is not None:
            self.model = model.to(self.device)
        if self.model is not None:
            self.model.eval()
            if hasattr(self.model, "set_precision"):
                self.model.set_precision("bf16" if self.use_half else "fp32")
        self.inference_times: deque = deque(maxlen=100)
        self.memory_usage: deque = deque(maxlen=100)
        self.stability_metrics: List[Dict[str, Any]] = []
        self.batch_queue: queue.Queue = queue.Queue(maxsize=config.max_batch_size)
        self.batch_thread: Optional[threading.Thread] = None
        self.batch_running = False
        self._lock = threading.Lock()
        self._runner = None
        if config.warmup_iterations > 0 and self.model is not None:
            self._warmup()

    # ------------------------------------------------------------------ setup
    def _load_model(self):
        ckpt = torch.load(self.config.model_path, map_location="cpu", weights_only=True)
        sd = ckpt.get("model_state_dict", ckpt.get("state_dict", ckpt)) if isinstance(ckpt, dict) else None
        if self.model is None or sd is None:
            raise RuntimeError("InferenceEngine: pass a model instance; checkpoints load as state_dicts only")
        self.model.load_state_dict(sd)
        self.model = self.model.to(self.device).eval()

    def _warmup(self):
        x = torch.randn(self.config.batch_size, 3, self.config.input_height, self.config.input_width,
                        device=self.device)
        with torch.no_grad():
            for _ in range(self.config.warmup_iterations):
                self.model(x, task="detection")
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        if self.config.use_graphs and hasattr(self.model, "capture"):
            self.model.freeze(True)
            self._runner = self.model.capture(x[:1].contiguous())

    def _to_tensor(self, image: Union[np.ndarray, torch.Tensor]) -> torch.Tensor:
        if isinstance(image, np.ndarray):
            return preprocess_image(image, self.config.input_height, self.config.input_width, self.device,
                                    resample=self.config.resample)
        return image.to(self.device)

    def preprocess_batch(self, images: List[np.ndarray]) -> torch.Tensor:
        if all(isinstance(i, np.ndarray) for i in images) and len({i.shape for i in images}) == 1:
            return preprocess_frames(images, self.config.input_height, self.config.input_width, self.device,
                                     resample=self.config.resample)
        return torch.stack([self._to_tensor(i) for i in images])

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def infer(self, image: Union[np.ndarray, torch.Tensor]) -> Dict[str, Any]:
        """engine.py:251-317."""
        start = time.perf_counter()
        x = self._to_tensor(image)
        if x.dim() == 3:
            x = x.unsqueeze(0)
        with self._lock:
            if self._runner is not None and tuple(x.shape) == tuple(self._runner.static_in.shape):
                outputs = self._runner(x, owned=True)
            else:
                outputs = self.model(x, task="detection")
            if self.device.type == "cuda":
                torch.cuda.synchronize()
        ms = (time.perf_counter() - start) * 1e3
        self.inference_times.append(ms)
        if self.device.type == "cuda":
            self.memory_usage.append(torch.cuda.memory_allocated() / 1024 ** 2)
        st = LazyStabilityMetrics(self.model)
        res = {"outputs": outputs, "inference_time_ms": ms, "batch_size": x.shape[0],
               "input_shape": x.shape, "device": str(self.device), "stability_metrics": st}
        if self.config.collect_stability:
            self.stability_metrics.append(dict(st))
        return res

    inference = infer   # call-site alias (scripts/inference.py:121)

    @torch.no_grad()
    def infer_batch(self, images: List[Union[np.ndarray, torch.Tensor]]) -> List[Dict[str, Any]]:
        """engine.py:319-387."""
        t0 = time.perf_counter()
        batch = torch.stack([self._to_tensor(i) for i in images])
        with self._lock:
            outputs = self.model(batch, task="detection")
            if self.device.type == "cuda":
                torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        results = []
        for i in range(len(images)):
            per = {}
            for k, v in outputs.items():
                if isinstance(v, torch.Tensor):
                    per[k] = v[i:i + 1]
                elif isinstance(v, dict):
                    per[k] = {kk: (vv[i:i + 1] if isinstance(vv, torch.Tensor) else vv) for kk, vv in v.items()}
                else:
                    per[k] = v
            results.append({"outputs": per, "batch_index": i, "batch_inference_time_ms": ms / len(images),
                            "total_inference_time_ms": ms})
        return results

    # ------------------------------------------------------------------ async (engine.py:389-471)
    def start_async_inference(self):
        if self.batch_thread is not None:
            logger.warning("Async inference already running")
            return
        self.batch_running = True
        self.batch_thread = threading.Thread(target=self._async_loop, daemon=True)
        self.batch_thread.start()

    def stop_async_inference(self):
        self.batch_running = False
        if self.batch_thread:
            self.batch_thread.join(timeout=5.0)
            self.batch_thread = None

    def _async_loop(self):
        buf, stamps = [], []
        while self.batch_running:
            try:
                item = self.batch_queue.get(timeout=0.1)
                buf.append(item)
                stamps.append(time.time())
            except queue.Empty:
                if not buf:
                    continue
            ready = len(buf) >= self.config.batch_size or (buf and time.time() - stamps[0] > 0.033)
            if ready:
                try:
                    for r, it in zip(self.infer_batch([b["image"] for b in buf]), buf):
                        if it.get("callback"):
                            it["callback"](r)
                except Exception as e:  # noqa: BLE001 -- the reference logs and keeps serving
                    logger.error(f"Error in async inference loop: {e}")
                buf.clear()
                stamps.clear()

    def async_infer(self, image: np.ndarray, callback: Optional[Callable] = None):
        if not self.batch_running:
            raise RuntimeError("Async inference not started")
        self.batch_queue.put({"image": image, "callback": callback, "timestamp": time.time()})

    # ------------------------------------------------------------------ stats (engine.py:473-562)
    def get_performance_stats(self) -> Dict[str, Any]:
        if not self.inference_times:
            return {}
        t = list(self.inference_times)
        stats = {"inference_time": {"mean": float(np.mean(t)), "std": float(np.std(t)), "min": float(np.min(t)),
                                    "max": float(np.max(t)), "p95": float(np.percentile(t, 95)),
                                    "p99": float(np.percentile(t, 99)), "latest": t[-1]},
                 "throughput_fps": 1000.0 / float(np.mean(t)), "total_inferences": len(t)}
        if self.memory_usage:
            m = list(self.memory_usage)
            stats["memory_usage_mb"] = {"mean": float(np.mean(m)), "max": float(np.max(m)), "current": m[-1]}
        stats["latency_constraint_met"] = stats["inference_time"]["p95"] <= self.config.max_latency_ms
        return stats

    def get_stability_report(self) -> Dict[str, Any]:
        if not self.stability_metrics:
            return {}
        rep = {"eigenvalues": [], "signal_ratios": [], "gradient_norms": [],
               "total_checks": len(self.stability_metrics)}
        for m in self.stability_metrics[-100:]:
            rep["eigenvalues"] += [v for k, v in m.items() if k.endswith("max_eigenvalue")]
            rep["signal_ratios"] += [v for k, v in m.items() if k.endswith("signal_ratio_mean")]
        if rep["eigenvalues"]:
            e = rep["eigenvalues"]
            rep["eigenvalue_stats"] = {"mean": float(np.mean(e)), "std": float(np.std(e)), "max": float(np.max(e))}
            rep["is_stable"] = all(v <= 1.0 + 1e-3 for v in e)
        if rep["signal_ratios"]:
            rep["signal_ratio_stats"] = {"mean": float(np.mean(rep["signal_ratios"])),
                                         "std": float(np.std(rep["signal_ratios"]))}
        return rep

    def reset_stats(self):
        self.inference_times.clear()
        self.memory_usage.clear()
        self.stability_metrics.clear()


class StreamingPipeline:
    """Camera-to-detections path of config E (the reference's per-frame loop is
    scripts/inference.py:224-291 -> process_image_frame: ImagePreprocessor.process, engine
    infer, DetectionPostprocessor, at 1280x720 / 30 FPS): one host->device copy of the raw
    uint8 BGR frame, then ONE hipGraph replay holding the Pillow-exact preprocessing
    (hv_preprocess_pil, written straight into the model's NHWC input), the whole forward with
    the coefficients frozen, the decode and the batched NMS (hv_nms), then one small
    device->host copy of the detections.

    Weights changed in place after capture (VersionWatch) trigger a re-capture before the
    frame's result is read, as in GraphRunner."""

    def __init__(self, model, frame_hw, input_hw=(640, 640), conf_threshold: float = 0.25,
                 iou_threshold: float = 0.45, max_detections: int = 100, resample: str = "pil"):
        self.model = model.eval()
        self.model.freeze(True)
        dev = next(model.parameters()).device
        self.dtype = PRECISION_DTYPES[getattr(model, "hv_precision", "bf16")]
        h, w = frame_hw
        H, W = input_hw
        self.frame_hw, self.input_hw, self.resample = (h, w), (H, W), resample
        self.nms_args = (conf_threshold, iou_threshold, max_detections)
        self.staging = torch.empty((1, h, w, 3), dtype=torch.uint8).pin_memory()
        self.frame = torch.empty((1, h, w, 3), dtype=torch.uint8, device=dev)
        self.inp = torch.empty((1, H, W, 3), dtype=self.dtype, device=dev)
        md = max_detections
        self.host = {"boxes": torch.empty((md, 4), dtype=torch.float32).pin_memory(),
                     "scores": torch.empty(md, dtype=torch.float32).pin_memory(),
                     "labels": torch.empty(md, dtype=torch.int64).pin_memory(),
                     "count": torch.empty(1, dtype=torch.int32).pin_memory()}
        self.recaptures = 0
        self._capture()

    def _forward(self):
        """-> (outputs, the RunCtx the forward ran under)."""
        H, W = self.input_hw
        x = ops.preprocess(self.frame, H, W, bgr=True, dtype=self.dtype, nhwc=True, out=self.inp,
                           resample=self.resample)
        return self.model.forward_eval(x, task="detection")

    def _capture(self):
        """Graph 1: preprocess + forward + decode.  The NMS plan's device table is then built
        (outside any capture) on graph 1's static decoded outputs, and graph 2 records its two
        launches."""
        self.graph = self.nms_graph = None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.no_grad():
            for _ in range(2):
                out = self._forward()[0]
                ops.NmsPlan(out["decoded"], *self.nms_args).run()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        del out
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"), torch.no_grad():
            # ctx: the buffers graph 1 reads outside its pool, pinned (detect.GraphRunner)
            self.outputs, self.ctx = self._forward()
        self._nms = ops.NmsPlan(self.outputs["decoded"], *self.nms_args)
        torch.cuda.synchronize()
        self.nms_graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.nms_graph):
            self.dets = self._nms.run()
        self.version = self.model._watch.snapshot()

    def __call__(self, frame: np.ndarray) -> Dict[str, np.ndarray]:
        """uint8 HWC BGR frame -> {'boxes' [k, 4] xyxy normalised, 'scores' [k], 'labels' [k]}."""
        if frame.shape != (*self.frame_hw, 3) or frame.dtype != np.uint8:
            raise ValueError(f"expected a uint8 {self.frame_hw + (3,)} frame")
        if self.model._watch.snapshot() != self.version:   # before any replay: no stale storage
            self.recaptures += 1
            self._capture()
        self.staging[0].numpy()[...] = frame
        self.frame.copy_(self.staging, non_blocking=True)
        self.graph.replay()
        self.nms_graph.replay()
        boxes, scores, labels, count = self.dets
        self.host["count"].copy_(count, non_blocking=True)
        self.host["boxes"].copy_(boxes[0], non_blocking=True)
        self.host["scores"].copy_(scores[0], non_blocking=True)
        self.host["labels"].copy_(labels[0], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        k = int(self.host["count"][0])
        return {"boxes": self.host["boxes"][:k].numpy().copy(), "scores": self.host["scores"][:k].numpy().copy(),
                "labels": self.host["labels"][:k].numpy().copy()}


class AsyncInferenceEngine(InferenceEngine):
    """engine.py:564-671: asyncio front-end over a thread pool (kernels are stream-ordered and
    the engine serialises model calls, so concurrent requests are safe)."""

    def __init__(self, config: Optional[InferenceConfig] = None, model: Optional[torch.nn.Module] = None, **kw):
        super().__init__(config, model, **kw)
        self.executor = ThreadPoolExecutor(max_workers=4)
        self.request_counter = 0

    async def infer_async(self, image: np.ndarray) -> Dict[str, Any]:
        self.request_counter += 1
        loop = asyncio.get_event_loop()
        return await loop.run_in_executor(self.executor, self.infer, image)

    def infer_sync(self, image: np.ndarray) -> Dict[str, Any]:
        try:
            loop = asyncio.get_event_loop()
        except RuntimeError:
            loop = asyncio.new_event_loop()
            asyncio.set_event_loop(loop)
        return loop.run_until_complete(self.infer_async(image))
