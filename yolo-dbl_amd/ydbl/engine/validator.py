"""Detection validation (mAP) over an in-memory dataset, for the mAP@0.5 acceptance check.

Follows BaseValidator.__call__ (U/engine/validator.py:107-220) and DetectionValidator
(U/models/yolo/detect/val.py:50-227) for tensor sources: NMS with multi_label=True at conf 0.001,
iou 0.7 (val.py:92-102) — run on the GPU in the same hipGraph as the forward —, boxes clipped
(scale_boxes with gain 1 / pad 0), TP matrix at IoU 0.5:0.95 (val.py:209-227 + match_predictions),
then ap_per_class.

A dataset is an iterable of batches ``{"img": float [B,3,H,W] (0..1 or 0..255), "cls": [N],
"bboxes": [N,4] xyxy pixels of the input image, "batch_idx": [N]}``.  LetterBox/letterboxed
file datasets are SURVEY §8f "next" (cv2 is not part of this path).
"""

from __future__ import annotations

import numpy as np
import torch

from ..utils.metrics import IOUV, DetMetrics, box_iou, match_predictions
from .model import load_tensor_source, select_device


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
            det, cnt = s(im)
            det, cnt = det.cpu(), cnt.cpu().tolist()
            bidx = torch.as_tensor(batch["batch_idx"]).cpu()
            cls_all = torch.as_tensor(batch["cls"]).cpu().float().reshape(-1)
            box_all = torch.as_tensor(batch["bboxes"]).cpu().float().reshape(-1, 4)
            for si in range(b):
                pred = det[si, : cnt[si]]
                sel = bidx == si
                cls, bbox = cls_all[sel], box_all[sel]
                nl, npr = len(cls), len(pred)
                tp = torch.zeros(npr, len(self.iouv), dtype=torch.bool)
                if npr == 0:
                    if nl:
                        stats["tp"].append(tp)
                        stats["conf"].append(torch.zeros(0))
                        stats["pred_cls"].append(torch.zeros(0))
                        stats["target_cls"].append(cls)
                    continue
                if self.args.get("single_cls", False):
                    pred[:, 5] = 0
                if nl:
                    tp = match_predictions(pred[:, 5], cls, box_iou(bbox, pred[:, :4]), self.iouv)
                stats["tp"].append(tp)
                stats["conf"].append(pred[:, 4])
                stats["pred_cls"].append(pred[:, 5])
                stats["target_cls"].append(cls)
        st = {k: torch.cat(v, 0).numpy() if v else np.zeros((0, 10) if k == "tp" else 0) for k, v in stats.items()}
        if len(st["tp"]) and st["tp"].any():
            self.metrics.process(st["tp"], st["conf"], st["pred_cls"], st["target_cls"])
        return self.metrics
