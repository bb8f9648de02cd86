"""User API: ``YOLO(cfg_or_weights)`` with ``.predict()``, ``.val()``, ``.fuse()``.

Mirrors U/engine/model.py:84-643 and U/models/yolo/model.py:52-100 for the
detect task: model files named like the reference's
(``yolov13n_DBL.yaml`` / ``yolov13s_DBL.yaml`` / ``yolov13l_DBL2.yaml``) build
the same layer graph; ``predict`` keeps the reference's argument names and
defaults (conf 0.25, iou 0.7, max_det 300, half False, agnostic_nms, classes;
U/cfg/default.yaml:51-54 and U/engine/model.py:547) and returns ``Results``.
Everything after construction runs on the GPU through libydbl; there is no CPU
execution path (``device='cpu'`` raises).
"""

from __future__ import annotations

import time
from collections import OrderedDict
from pathlib import Path

import numpy as np
import torch

from ..nn.tasks import DetectionModel, weights_signature, ydbl_env
from .results import Results
from .session import DetectSession, default_streams

DEFAULTS = {"conf": 0.25, "iou": 0.7, "max_det": 300, "half": False, "fp8": False, "device": None, "agnostic_nms": False,
            "classes": None, "batch": 1, "verbose": False, "imgsz": 640,
            # sub-batch graphs per session (DetectSession): None = default_streams(batch), the benched layout
            "streams": None,
            # fp8: an ydbl.quant.Fp8Calibration or its JSON file (None: calibrate on the first batch)
            "fp8_calibration": None}


def select_device(device=None) -> torch.device:
    """U/utils/torch_utils.py select_device, GPU-only."""
    if device is None or device == "":
        device = 0
    if isinstance(device, torch.device):
        dev = device
    elif isinstance(device, int):
        dev = torch.device("cuda", device)
    else:
        s = str(device).lower().replace("cuda:", "").strip()
        if s == "cpu":
            raise RuntimeError("ydbl runs on MI355X (gfx950) only; device='cpu' has no implementation")
        dev = torch.device("cuda", int(s.split(",")[0]) if s else 0)
    if dev.type != "cuda":
        raise RuntimeError(f"ydbl runs on MI355X (gfx950) only; got device {dev}")
    if not torch.cuda.is_available():
        raise RuntimeError("no GPU visible: ydbl has no CPU fallback")
    return dev


def load_tensor_source(im: torch.Tensor, stride: int = 32) -> torch.Tensor:
    """LoadTensor._single_check (U/data/loaders.py:515-580): BCHW, H and W divisible by the stride, /255 if >1."""
    im = check_tensor_source(im, stride)
    if im.max() > 1.0 + torch.finfo(im.dtype).eps:
        im = im.float() / 255.0
    return im


def check_tensor_source(im, stride: int = 32) -> torch.Tensor:
    """The shape rules of LoadTensor._single_check (no device work): a BCHW tensor (or a list of CHW / 1CHW)."""
    if isinstance(im, (list, tuple)):
        im = torch.stack([t if t.ndim == 3 else t[0] for t in im])
    if not isinstance(im, torch.Tensor):
        raise TypeError(f"ydbl predict() takes torch tensors (BCHW float); got {type(im).__name__}")
    if im.ndim == 3:
        im = im.unsqueeze(0)
    if im.ndim != 4 or im.shape[1] != 3:
        raise ValueError(f"torch.Tensor inputs should be BCHW i.e. shape(b, 3, h, w) but got {tuple(im.shape)}")
    if im.shape[2] % stride or im.shape[3] % stride:
        raise ValueError(
            f"torch.Tensor inputs should be BCHW with height and width divisible by stride {stride}; got {tuple(im.shape)}")
    return im


_SCALES = {}


def _calib_key(cal):
    """Session-cache key of an fp8 calibration: its path, or a fingerprint of its content (not id(): a new object
    for the same record would compile a new session, and a recycled id could hit a session of another record)."""
    if cal is None or isinstance(cal, (str, Path)):
        return None if cal is None else str(cal)
    fp = getattr(cal, "_ydbl_fingerprint", None)
    if fp is None:
        import hashlib
        import json

        fp = hashlib.sha1(json.dumps(cal.to_json(), sort_keys=True).encode()).hexdigest()
        try:
            cal._ydbl_fingerprint = fp
        except AttributeError:
            pass
    return fp


def _scale_consts(dev):
    """(1.0, fp32(1/255)) as 0-dim fp32 tensors on `dev` (made once)."""
    c = _SCALES.get(dev)
    if c is None:
        c = _SCALES[dev] = (torch.ones((), dtype=torch.float32, device=dev),
                            torch.full((), 1.0 / 255.0, dtype=torch.float32, device=dev))
    return c


class _LazyHWC:
    """Per-image HWC views of a batch, scaled by a 0-dim device tensor, made on first access (Results.orig_img)."""

    def __init__(self, im, scale):
        self.im, self.scale, self.hwc = im, scale, None

    def __getitem__(self, i):
        if self.hwc is None:
            scale = self.scale() if callable(self.scale) else self.scale
            x = self.im.float() if scale is None else self.im.float() * scale
            self.hwc = x.permute(0, 2, 3, 1)
        return self.hwc[i]


class _LazyCounts:
    """The per-image detection counts of a batch, read to the host once, on first access: predict() returns without
    waiting for the GPU, and the batch's Results synchronise when one of them is first looked at.  cnt: the device
    tensor, or a callable producing it then (a session slot's outputs, copied out on first access)."""

    def __init__(self, cnt):
        self.cnt, self.host = cnt, None

    def __getitem__(self, i):
        if self.host is None:
            self.host = (self.cnt() if callable(self.cnt) else self.cnt).tolist()
        return self.host[i]


class Model:
    """U/engine/model.py:84-643 (detect task subset)."""

    def __init__(self, model: str | Path = "yolov13n_DBL.yaml", task=None, verbose=False, nc=None):
        self.task = task or "detect"
        self.overrides = {}
        self.ckpt_path = None
        self.verbose = verbose
        self._sessions = OrderedDict()  # LRU of compiled sessions (each holds its own HBM buffers)
        model = str(model)
        suffix = Path(model).suffix.lower()
        if suffix in (".pt", ".pth"):
            # reference checkpoint: build from its embedded yaml, then load its weights (U/nn/tasks.py:921-944)
            from ..utils.checkpoint import read_reference_checkpoint

            ck = read_reference_checkpoint(model)
            if ck["yaml"] is None:
                raise ValueError(f"{model} has no embedded model yaml: build from a config and call .load()")
            self.model = DetectionModel(ck["yaml"], nc=nc, verbose=verbose)
            self._load_sd(ck["state_dict"])
            if ck["names"]:
                self.model.names = ck["names"]
            self.ckpt_path = model
        elif suffix == ".safetensors":
            raise ValueError("build from a config and call .load(weights): YOLO('yolov13n_DBL.yaml').load('w.safetensors')")
        else:
            self.model = DetectionModel(model, nc=nc, verbose=verbose)
        self.cfg = model
        self.overrides["model"] = model

    # ------------------------------------------------------------------ weights
    def load(self, weights):
        """Load a state_dict (torch weights_only file, safetensors, or a dict) with the reference's key names."""
        names = None
        if isinstance(weights, dict):
            sd = weights
        elif str(weights).endswith(".safetensors"):
            from safetensors.torch import load_file

            sd = load_file(str(weights))
        else:
            # plain state_dict files and the reference trainer's checkpoints, both without executing code
            from ..utils.checkpoint import read_reference_checkpoint

            ck = read_reference_checkpoint(weights)
            sd, names = ck["state_dict"], ck["names"]
        self._load_sd(sd)
        if names:
            self.model.names = names
        self.ckpt_path = str(weights) if not isinstance(weights, dict) else None
        return self

    def _load_sd(self, sd):
        sd = {k[len("model."):] if k.startswith("model.model.") else k: v for k, v in sd.items()}
        missing, unexpected = self.model.load_state_dict(sd, strict=False)
        if unexpected:
            raise KeyError(f"unexpected keys in weights: {unexpected[:5]} ...")
        # BN's num_batches_tracked counter carries no weight (the reference's checkpoints may omit it);
        # every other parameter/buffer must be present: a partial dict would leave layers at random init
        missing = [k for k in missing if not k.endswith("num_batches_tracked")]
        if missing:
            raise KeyError(f"{len(missing)} keys missing from weights: {missing[:5]} ...")
        self._sessions.clear()

    def state_dict(self):
        return self.model.state_dict()

    @property
    def names(self):
        return self.model.names

    @property
    def stride(self):
        return self.model.stride

    def fuse(self):
        self.model.fuse()
        return self

    def info(self):
        n = sum(p.numel() for p in self.model.parameters())
        return {"layers": len(self.model.model), "parameters": n}

    # ------------------------------------------------------------------ inference
    MAX_SESSIONS = 4  # a DBL-n bs32 640 fp16 session holds ~0.95 GB of HBM: keep the few most recently used

    def session(self, batch, h, w, half=False, conf=0.25, iou=0.7, max_det=300, agnostic=False, classes=None,
                multi_label=False, device=None, keep_pred=False, use_graph=True, fp8=False, clip=True,
                streams=1, gather_rows=None, nms=True, fp8_calibration=None) -> DetectSession:
        """A compiled (batch, h, w, dtype, NMS settings) inference session; streams > 1 splits the batch into
        that many concurrently replayed sub-batch graphs (DetectSession); streams=None: default_streams(batch),
        the layout predict() runs and bench.py times."""
        if streams is None:
            streams = default_streams(batch)
        dev = select_device(device)
        dtype = torch.float16 if (half or fp8) else torch.float32
        key = (batch, h, w, dtype, float(conf), float(iou), int(max_det), bool(agnostic),
               tuple(classes) if classes is not None else None, bool(multi_label), str(dev), keep_pred, use_graph,
               float(fp8), bool(clip), int(streams), gather_rows, bool(nms),
               _calib_key(fp8_calibration),
               # the remaining YDBL_* switches (plan-builder fusions in ydbl.nn.modules; YDBL_DS_LEAN / YDBL_NMS_*
               # in the C-ABI) are read at plan build or at each launch, so a captured graph keeps the routing of
               # its capture: a different switch setting is a different session
               ydbl_env())
        s = self._sessions.get(key)
        if s is None:
            while len(self._sessions) >= self.MAX_SESSIONS:
                self._sessions.popitem(last=False)  # least recently used; its buffers go with the last reference
            with torch.cuda.device(dev):
                s = DetectSession(self.model, batch, h, w, dtype, conf, iou, max_det, multi_label, agnostic, classes,
                                  keep_pred=keep_pred, use_graph=use_graph, device=dev, fp8=fp8, clip=clip,
                                  streams=streams, gather_rows=gather_rows, nms=nms, fp8_calibration=fp8_calibration)
            s.wsig = weights_signature(self.model)  # the weights its plans folded (see _stale)
            self._sessions[key] = s
        else:
            self._sessions.move_to_end(key)
        return s

    def reset_sessions(self):
        """Drop every compiled session (after editing weights through ``.data``, which no signature sees)."""
        self._sessions.clear()
        self.model.invalidate()
        return self

    def _stale(self, s) -> bool:
        """True (and `s` dropped from the cache) when the weights changed since `s` folded them (in-place edits,
        replaced tensors: nn.tasks.weights_signature).  Called right after a launch, so the ~90 us check runs
        while the graph does."""
        if weights_signature(self.model) == s.wsig:
            return False
        for k in [k for k, v in self._sessions.items() if v is s]:
            del self._sessions[k]
        return True

    def predict(self, source=None, stream=False, **kwargs):
        """U/engine/model.py:501-560 + DetectionPredictor.postprocess (U/models/yolo/detect/predict.py:23-41).

        source (ydbl.engine.sources, after load_inference_source U/data/build.py:182-215):
          - BCHW float tensor (LoadTensor rules): run as given;
          - PIL image(s), HWC uint8 BGR ndarray frame(s), or a list of image paths (LoadPilAndNumpy): one batch;
          - str / Path: an image file, a directory, a glob or a *.txt list (LoadImagesAndVideos): batches of
            ``batch`` images (default 1) in sorted file order.
        Non-tensor sources are letterboxed to imgsz on the GPU and their boxes come back in the original
        image's coordinates.
        """
        from .sources import check_path_source, file_batches, frames_from_images, is_frame_source

        args = {**DEFAULTS, **self.overrides, **kwargs}
        dev = select_device(args["device"])
        t0 = time.perf_counter()
        if source is None:
            raise ValueError("predict() needs a source (no default asset is bundled)")
        if not isinstance(source, torch.Tensor) and not (isinstance(source, (list, tuple)) and source
                                                         and isinstance(source[0], torch.Tensor)):
            if check_path_source(source):
                gen = (r for paths, frames in file_batches(source, args["batch"])
                       for r in self._predict_frames(frames, args, dev, time.perf_counter(), False, paths))
                return gen if stream else list(gen)
            if is_frame_source(source):
                paths, frames = frames_from_images(source)
                return self._predict_frames(frames, args, dev, t0, stream, paths)
            raise TypeError(f"unsupported source type {type(source).__name__}")
        im = check_tensor_source(source, int(self.model.stride.max()))
        if im.device != dev:  # host tensors are scaled on the host, where the reference's LoadTensor does it, then moved
            im = load_tensor_source(im).to(dev, non_blocking=True).float()
        b, _, h, w = im.shape
        kw = dict(half=args["half"], conf=args["conf"], iou=args["iou"], max_det=args["max_det"],
                  agnostic=args["agnostic_nms"], classes=args["classes"], device=dev, fp8=args["fp8"],
                  streams=args["streams"], fp8_calibration=args["fp8_calibration"])
        s = self.session(b, h, w, **kw)
        t1 = time.perf_counter()
        one, inv = _scale_consts(dev)
        thr = 1.0 + (torch.finfo(im.dtype).eps if im.is_floating_point() else 0.0)
        bo = None
        if s.can_bind(im):
            # read in place: the plans' input binding points at im, and the stem kernels apply LoadTensor's /255
            # rule from its device-side maximum (no staging copy, no host sync, no per-call copy of the outputs;
            # DetectSession.launch_bound)
            bo = s.launch_bound(im)
        else:
            # LoadTensor's /255 rule on the device without a host sync: the input copy multiplies by fp32(1/255)
            # when max > 1 (torch's GPU x / 255.0 is exactly that product), by 1 otherwise
            scale = torch.where(im.amax() > thr, inv, one)
            det, cnt = s(im, scale)
        if self._stale(s):  # weights edited since the session was compiled: rebuild and run again
            s = self.session(b, h, w, **kw)
            scale = torch.where(im.amax() > thr, inv, one)
            (det, cnt), bo = s(im, scale), None
        # no host sync here: each image's boxes are a view of the batch's det, cut at its count when first accessed
        # (_LazyCounts: one sync for the batch) -- on the copy path one device copy of det | count made now (the
        # session's buffers are reused by the next call); orig_img a view of the input batch (HWC, as LoadTensor
        # hands it over), made on first access.  speed["inference"] is the launch time.
        if bo is not None:  # the slot's outputs, copied out of the slot on first access (or when it is reused)
            dets, counts, scale = None, _LazyCounts(lambda: bo.detach().count), (lambda: bo.detach().scale[0])
        elif getattr(s, "out_flat", None) is not None:  # det | count: one copy
            flat = s.out_flat.clone()
            dets, counts = flat[: det.numel()].view(det.shape), _LazyCounts(flat[det.numel():].view(torch.int32))
        else:
            dets, counts = det.clone(), _LazyCounts(cnt.clone())
        t2 = time.perf_counter()
        speed = {"preprocess": (t1 - t0) * 1e3 / b, "inference": (t2 - t1) * 1e3 / b, "postprocess": 0.0}
        hwc = _LazyHWC(im, scale)
        names, shape = self.model.names, (h, w)
        if bo is not None:
            box = lambda i: bo.detach().det[i, : counts[i]]  # noqa: E731
        else:
            box = lambda i: dets[i, : counts[i]]  # noqa: E731
        results = [Results(lambda i=i: hwc[i], path=f"image{i}.jpg", names=names, speed=speed, orig_shape=shape,
                           boxes=lambda i=i: box(i)) for i in range(b)]
        return iter(results) if stream else results

    def _predict_frames(self, frames, args, dev, t0, stream, paths=None):
        from .preprocess import letterbox_batch, scale_boxes

        frames = [frames] if isinstance(frames, np.ndarray) and frames.ndim == 3 else list(frames)
        imgsz = args["imgsz"]
        imgsz = (imgsz, imgsz) if isinstance(imgsz, int) else tuple(imgsz)
        stride = int(self.model.stride.max())
        im = letterbox_batch(frames, imgsz, stride=stride, device=dev)
        b, _, h, w = im.shape
        # the reference's NMS does not clip: boxes are clipped to the frame by scale_boxes
        s = self.session(b, h, w, half=args["half"], conf=args["conf"], iou=args["iou"], max_det=args["max_det"],
                         agnostic=args["agnostic_nms"], classes=args["classes"], device=dev, fp8=args["fp8"],
                         clip=False, streams=args["streams"], fp8_calibration=args["fp8_calibration"])
        t1 = time.perf_counter()
        det, cnt = s(im)
        if self._stale(s):
            det, cnt = self.session(b, h, w, half=args["half"], conf=args["conf"], iou=args["iou"],
                                    max_det=args["max_det"], agnostic=args["agnostic_nms"], classes=args["classes"],
                                    device=dev, fp8=args["fp8"], clip=False, streams=args["streams"],
                                    fp8_calibration=args["fp8_calibration"])(im)
        counts = cnt.tolist()
        t2 = time.perf_counter()
        results = []
        for i, f in enumerate(frames):
            boxes = det[i, : counts[i]].clone()
            scale_boxes((h, w), boxes, f.shape[:2])
            results.append(Results(f, path=paths[i] if paths else f"image{i}.jpg", names=self.model.names,
                                   boxes=boxes))
        t3 = time.perf_counter()
        speed = {"preprocess": (t1 - t0) * 1e3 / b, "inference": (t2 - t1) * 1e3 / b,
                 "postprocess": (t3 - t2) * 1e3 / b}
        for r in results:
            r.speed = speed
        return iter(results) if stream else results

    __call__ = predict

    def val(self, data=None, **kwargs):
        """Detection mAP (U/engine/model.py:609-643): ``data`` = a data YAML, a dataset folder, an image folder /
        list, or in-memory batches; see ydbl.engine.validator.  rect batches by default, like the reference."""
        from .validator import DetectionValidator

        args = {**DEFAULTS, "conf": 0.001, "iou": 0.7, "batch": 16, "rect": True, "split": "val", **kwargs}
        return DetectionValidator(self, args)(data)


class YOLO(Model):
    """U/models/yolo/model.py:52-100 — detect task only."""

    @property
    def task_map(self):
        return {"detect": {"model": DetectionModel, "predictor": DetectSession}}
