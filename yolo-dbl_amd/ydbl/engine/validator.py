"""Detection validation (mAP) for the mAP@0.5 acceptance check.

Follows BaseValidator.__call__ (U/engine/validator.py:107-220) and DetectionValidator
(U/models/yolo/detect/val.py:50-227): NMS with multi_label=True at conf 0.001, iou 0.7 (val.py:92-102) —
run on the GPU in the same hipGraph as the forward —, TP matrix at IoU 0.5:0.95 (val.py:209-227 +
match_predictions) on the device with ydbl_match_predictions right behind NMS, then ap_per_class on the host.

``data`` is either
- a data YAML / its folder / its parsed dict (check_det_dataset), or an image directory / *.txt list: a
  YOLO-format dataset read by ydbl.engine.dataset (rect batches, letterboxed on the GPU by ydbl_letterbox) and
  matched in native image space after scale_boxes(ratio_pad) (val.py:104-123), like the reference; or
- an iterable of in-memory batches ``{"img": float [B,3,H,W] (0..1 or 0..255), "cls": [N], "bboxes": [N,4]
  xyxy pixels of the input image, "batch_idx": [N]}`` (boxes clipped to the input, gain 1 / pad 0).
"""

from __future__ import annotations

import ctypes as C
import math
import os
from pathlib import Path

import numpy as np
import torch

from .. import _lib
from ..utils.metrics import IOUV, DetMetrics
from .model import load_tensor_source, select_device


def match_batch(det: torch.Tensor, count: torch.Tensor, gt_box: torch.Tensor, gt_cls: torch.Tensor,
                batch_idx: torch.Tensor, iouv: torch.Tensor = IOUV, single_cls: bool = False) -> torch.Tensor:
    """TP matrix of one batch on the device (ydbl_match_predictions).

    det fp32 [B, max_det, 6] and count int32 [B] as NMS leaves them; labels gt_box [N, 4] xyxy,
    gt_cls [N], batch_idx [N] in any image order (kept in order within an image, like the
    reference's per-image label slice).  Returns bool [B, max_det, len(iouv)] on det's device;
    rows >= count are False.  Same results as DetectionValidator._process_batch
    (U/models/yolo/detect/val.py:209-227) per image.
    """
    if det.device.type != "cuda":
        raise RuntimeError("match_batch runs on the GPU (ydbl_match_predictions); got a CPU tensor")
    dev = det.device
    b, max_det = det.shape[0], det.shape[1]
    bidx = torch.as_tensor(batch_idx).reshape(-1).long().cpu()
    order = torch.argsort(bidx, stable=True)
    ofs = torch.zeros(b + 1, dtype=torch.int32)
    if len(bidx):
        if int(bidx.min()) < 0 or int(bidx.max()) >= b:
            raise ValueError(f"batch_idx must be in [0, {b})")
        ofs[1:] = torch.cumsum(torch.bincount(bidx, minlength=b), 0).to(torch.int32)
    n_gt = len(bidx)
    boxes = torch.as_tensor(gt_box).reshape(-1, 4).float().cpu()[order].to(dev).contiguous()
    cls = torch.as_tensor(gt_cls).reshape(-1).float().cpu()[order].to(dev).contiguous()
    ofs = ofs.to(dev)
    iouv_d = iouv.float().to(dev).contiguous()
    det = det.float().contiguous()
    count = count.to(dev, torch.int32).contiguous()
    out = torch.empty((b, max_det, len(iouv)), dtype=torch.uint8, device=dev)
    ws = torch.empty(int(_lib.lib.ydbl_match_workspace(b, max_det, n_gt, len(iouv))), dtype=torch.uint8, device=dev)
    d = _lib.MatchDesc(det.data_ptr(), count.data_ptr(), b, max_det, boxes.data_ptr() if n_gt else None,
                       cls.data_ptr() if n_gt else None, ofs.data_ptr(), n_gt, iouv_d.data_ptr(), len(iouv),
                       int(bool(single_cls)), out.data_ptr(), ws.data_ptr())
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(_lib.lib.ydbl_match_predictions(C.byref(d), stream), "ydbl_match_predictions")
    return out.bool()


class DetectionValidator:
    def __init__(self, model, args):
        self.model = model
        self.args = args
        self.iouv = IOUV
        self.metrics = DetMetrics(names=model.names)

    def __call__(self, data):
        if data is None:
            raise ValueError("val(data=...) needs a data YAML, an image folder, or an iterable of batches")
        dev = select_device(self.args.get("device"))
        self.stats = {"tp": [], "conf": [], "pred_cls": [], "target_cls": []}
        self.seen = 0
        if isinstance(data, (str, os.PathLike, dict)):
            self._run_dataset(data, dev)
        else:
            for batch in data:
                self._run_tensor_batch(batch, dev)
        st = {k: torch.cat(v, 0).numpy() if v else np.zeros((0, 10) if k == "tp" else 0) for k, v in self.stats.items()}
        if len(st["tp"]) and st["tp"].any():
            self.metrics.process(st["tp"], st["conf"], st["pred_cls"], st["target_cls"])
        return self.metrics

    def _session(self, b, h, w, dev, clip):
        a = self.args
        return self.model.session(b, h, w, half=a.get("half", False), conf=a["conf"], iou=a["iou"],
                                  max_det=a.get("max_det", 300), multi_label=True,
                                  agnostic=a.get("agnostic_nms", False) or a.get("single_cls", False), device=dev,
                                  fp8=a.get("fp8", False), clip=clip, streams=a.get("streams") or 1,
                                  fp8_calibration=a.get("fp8_calibration"))

    def _run_tensor_batch(self, batch, dev):
        im = load_tensor_source(batch["img"], int(self.model.model.stride.max())).to(dev).float()
        b, _, h, w = im.shape
        det_d, cnt_d = self._session(b, h, w, dev, clip=True)(im)
        self._update(det_d, cnt_d, torch.as_tensor(batch["bboxes"]).cpu().float().reshape(-1, 4),
                     torch.as_tensor(batch["cls"]).cpu().float().reshape(-1),
                     torch.as_tensor(batch["batch_idx"]).cpu().reshape(-1))

    def _run_dataset(self, data, dev):
        """A YOLO-format dataset: rect batches letterboxed on the GPU, predictions and labels in native space."""
        from .dataset import YOLOValDataset, check_det_dataset
        from .preprocess import letterbox_frames

        a = self.args
        stride = int(self.model.model.stride.max())
        names = self.model.names
        src = data
        is_yaml = isinstance(data, dict) or str(data).rsplit(".", 1)[-1] in {"yaml", "yml"} or (
            Path(data).is_dir() and (list(Path(data).glob("*.yaml")) or not _has_images(Path(data))))
        if is_yaml:
            info = check_det_dataset(data)
            src = info.get(a.get("split", "val"))
            if not src:
                raise FileNotFoundError(f"dataset has no '{a.get('split', 'val')}' split")
            num_cls = info["nc"]
        else:
            num_cls = len(names)
        imgsz = a.get("imgsz", 640)
        imgsz = imgsz if isinstance(imgsz, int) else max(imgsz)
        imgsz = max(math.ceil(imgsz / stride) * stride, stride)  # check_imgsz (U/utils/checks.py)
        ds = YOLOValDataset(src, imgsz=imgsz, batch_size=a.get("batch", 16), stride=stride, rect=a.get("rect", True),
                            single_cls=a.get("single_cls", False), classes=a.get("classes"), num_cls=num_cls,
                            workers=a.get("workers", 8))
        self.dataset = ds
        for hb in ds.batches():
            H, W = hb["shape"]
            b = len(hb["frames"])
            im = letterbox_frames(hb["frames"], hb["meta"], H, W, device=dev)
            # the reference's val NMS does not clip: scale_boxes clips to the original image afterwards
            det_d, cnt_d = self._session(b, H, W, dev, clip=False)(im)
            det_n = det_d.clone()
            gain = torch.tensor([rp[0][0] for rp in hb["ratio_pad"]], dtype=torch.float32, device=dev)
            pad = torch.tensor([rp[1] for rp in hb["ratio_pad"]], dtype=torch.float32, device=dev)
            ori = torch.tensor([[s[1], s[0]] for s in hb["ori_shape"]], dtype=torch.float32, device=dev)
            _scale_clip(det_n[..., :4], pad[:, None, :], gain[:, None, None], ori[:, None, :])
            bidx = torch.from_numpy(hb["batch_idx"]).long()
            native = native_labels(hb)
            self._update(det_n, cnt_d, native, torch.from_numpy(hb["cls"]).float(), bidx)

    def _update(self, det_d, cnt_d, box_all, cls_all, bidx):
        """update_metrics (val.py:125-172) for one batch: device TP matrix, host stats in image order."""
        b = det_d.shape[0]
        single = bool(self.args.get("single_cls", False))
        tp_all = match_batch(det_d, cnt_d, box_all, cls_all, bidx, self.iouv, single).cpu()
        det, cnt = det_d.cpu(), cnt_d.cpu().tolist()
        for si in range(b):
            self.seen += 1
            pred = det[si, : cnt[si]]
            cls = cls_all[bidx == si]
            nl, npr = len(cls), len(pred)
            if npr == 0:
                if nl:
                    self.stats["tp"].append(torch.zeros(0, len(self.iouv), dtype=torch.bool))
                    self.stats["conf"].append(torch.zeros(0))
                    self.stats["pred_cls"].append(torch.zeros(0))
                    self.stats["target_cls"].append(cls)
                continue
            if single:
                pred[:, 5] = 0
            self.stats["tp"].append(tp_all[si, :npr])
            self.stats["conf"].append(pred[:, 4])
            self.stats["pred_cls"].append(pred[:, 5])
            self.stats["target_cls"].append(cls)


def native_labels(hb) -> torch.Tensor:
    """A host batch's labels (normalized xywh of the letterboxed image) -> xyxy in original-image pixels:
    DetectionValidator._prepare_batch (U/models/yolo/detect/val.py:104-115) with scale_boxes(ratio_pad)
    (U/utils/ops.py:92-127), per image as the reference runs it, in fp32 torch ops."""
    H, W = hb["shape"]
    boxes = torch.from_numpy(hb["bboxes"]).reshape(-1, 4)
    bidx = torch.from_numpy(hb["batch_idx"]).long()
    native = torch.zeros_like(boxes)
    for si in range(len(hb["ori_shape"])):
        idx = bidx == si
        if idx.any():
            bb = _xywh2xyxy(boxes[idx]) * torch.tensor((W, H, W, H))
            (g0, _), (pw, ph) = hb["ratio_pad"][si]
            bb[:, 0] -= pw
            bb[:, 1] -= ph
            bb[:, 2] -= pw
            bb[:, 3] -= ph
            bb /= g0
            h0, w0 = hb["ori_shape"][si]
            bb[:, 0].clamp_(0, w0)
            bb[:, 1].clamp_(0, h0)
            bb[:, 2].clamp_(0, w0)
            bb[:, 3].clamp_(0, h0)
            native[idx] = bb
    return native


def _has_images(p: Path) -> bool:
    from .dataset import IMG_FORMATS

    return any(f.suffix[1:].lower() in IMG_FORMATS for f in p.rglob("*.*"))


def _xywh2xyxy(x: torch.Tensor) -> torch.Tensor:
    """U/utils/ops.py:416-433."""
    y = torch.empty_like(x)
    xy, wh = x[..., :2], x[..., 2:] / 2
    y[..., :2] = xy - wh
    y[..., 2:] = xy + wh
    return y


def _scale_clip(boxes: torch.Tensor, pad: torch.Tensor, gain: torch.Tensor, wh: torch.Tensor) -> None:
    """scale_boxes(ratio_pad) + clip_boxes (U/utils/ops.py:92-127, :319-338) for a padded [B, max_det, 4] block
    of device boxes, in place; pad [B, 1, 2] (x, y), gain [B, 1, 1], wh [B, 1, 2] original (w, h)."""
    boxes[..., 0:2] -= pad
    boxes[..., 2:4] -= pad
    boxes /= gain
    boxes[..., 0:2] = torch.minimum(boxes[..., 0:2].clamp(min=0), wh)
    boxes[..., 2:4] = torch.minimum(boxes[..., 2:4].clamp(min=0), wh)
