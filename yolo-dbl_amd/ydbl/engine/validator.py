"""Detection validation (mAP) over an in-memory dataset, for the mAP@0.5 acceptance check.

Follows BaseValidator.__call__ (U/engine/validator.py:107-220) and DetectionValidator
(U/models/yolo/detect/val.py:50-227) for tensor sources: NMS with multi_label=True at conf 0.001,
iou 0.7 (val.py:92-102) — run on the GPU in the same hipGraph as the forward —, boxes clipped
(scale_boxes with gain 1 / pad 0), TP matrix at IoU 0.5:0.95 (val.py:209-227 + match_predictions)
on the device with ydbl_match_predictions right behind NMS, then ap_per_class on the host.

A dataset is an iterable of batches ``{"img": float [B,3,H,W] (0..1 or 0..255), "cls": [N],
"bboxes": [N,4] xyxy pixels of the input image, "batch_idx": [N]}``.  LetterBox/letterboxed
file datasets are SURVEY §8f "next" (cv2 is not part of this path).
"""

from __future__ import annotations

import ctypes as C

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
            raise ValueError("val(data=...) needs an in-memory dataset (iterable of batches); see ydbl.engine.validator")
        dev = select_device(self.args.get("device"))
        stats = {"tp": [], "conf": [], "pred_cls": [], "target_cls": []}
        for batch in data:
            im = load_tensor_source(batch["img"], int(self.model.model.stride.max())).to(dev).float()
            b, _, h, w = im.shape
            s = self.model.session(b, h, w, half=self.args.get("half", False), conf=self.args["conf"],
                                   iou=self.args["iou"], max_det=self.args.get("max_det", 300), multi_label=True,
                                   agnostic=self.args.get("agnostic_nms", False) or self.args.get("single_cls", False),
                                   device=dev, fp8=self.args.get("fp8", False))
            det_d, cnt_d = s(im)
            bidx = torch.as_tensor(batch["batch_idx"]).cpu().reshape(-1)
            cls_all = torch.as_tensor(batch["cls"]).cpu().float().reshape(-1)
            box_all = torch.as_tensor(batch["bboxes"]).cpu().float().reshape(-1, 4)
            single = bool(self.args.get("single_cls", False))
            tp_all = match_batch(det_d, cnt_d, box_all, cls_all, bidx, self.iouv, single).cpu()
            det, cnt = det_d.cpu(), cnt_d.cpu().tolist()
            for si in range(b):
                pred = det[si, : cnt[si]]
                cls = cls_all[bidx == si]
                nl, npr = len(cls), len(pred)
                if npr == 0:
                    if nl:
                        stats["tp"].append(torch.zeros(0, len(self.iouv), dtype=torch.bool))
                        stats["conf"].append(torch.zeros(0))
                        stats["pred_cls"].append(torch.zeros(0))
                        stats["target_cls"].append(cls)
                    continue
                if single:
                    pred[:, 5] = 0
                tp = tp_all[si, :npr]
                stats["tp"].append(tp)
                stats["conf"].append(pred[:, 4])
                stats["pred_cls"].append(pred[:, 5])
                stats["target_cls"].append(cls)
        st = {k: torch.cat(v, 0).numpy() if v else np.zeros((0, 10) if k == "tp" else 0) for k, v in stats.items()}
        if len(st["tp"]) and st["tp"].any():
            self.metrics.process(st["tp"], st["conf"], st["pred_cls"], st["target_cls"])
        return self.metrics
