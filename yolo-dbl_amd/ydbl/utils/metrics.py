"""Detection metrics for the mAP acceptance check (host numpy, as the reference computes them).

Restates U/utils/metrics.py:52-71 (box_iou), :447-452 (smooth), :505-534 (compute_ap, 101-point COCO
interpolation), :537-623 (ap_per_class), :808-896 (DetMetrics keys incl. mAP75) and
U/engine/validator.py:222-262 (match_predictions, greedy by IoU, unique label / detection).
"""

from __future__ import annotations

import numpy as np
import torch

IOUV = torch.linspace(0.5, 0.95, 10)  # U/models/yolo/detect/val.py:36 (iou vector for mAP@0.5:0.95)

_trapz = getattr(np, "trapezoid", None) or np.trapz


def box_iou(box1: torch.Tensor, box2: torch.Tensor, eps: float = 1e-7) -> torch.Tensor:
    """U/utils/metrics.py:52-71: pairwise IoU of xyxy boxes, [N, M]."""
    (a1, a2), (b1, b2) = box1.float().unsqueeze(1).chunk(2, 2), box2.float().unsqueeze(0).chunk(2, 2)
    inter = (torch.min(a2, b2) - torch.max(a1, b1)).clamp_(0).prod(2)
    return inter / ((a2 - a1).prod(2) + (b2 - b1).prod(2) - inter + eps)


def match_predictions(pred_classes: torch.Tensor, true_classes: torch.Tensor, iou: torch.Tensor,
                      iouv: torch.Tensor = IOUV) -> torch.Tensor:
    """U/engine/validator.py:222-262 (non-scipy branch). iou: [labels, detections]."""
    correct = np.zeros((pred_classes.shape[0], iouv.shape[0])).astype(bool)
    correct_class = true_classes[:, None] == pred_classes
    iou = (iou * correct_class).cpu().numpy()
    for i, threshold in enumerate(iouv.cpu().tolist()):
        matches = np.nonzero(iou >= threshold)
        matches = np.array(matches).T
        if matches.shape[0]:
            if matches.shape[0] > 1:
                matches = matches[iou[matches[:, 0], matches[:, 1]].argsort()[::-1]]
                matches = matches[np.unique(matches[:, 1], return_index=True)[1]]
                matches = matches[np.unique(matches[:, 0], return_index=True)[1]]
            correct[matches[:, 1].astype(int), i] = True
    return torch.tensor(correct, dtype=torch.bool, device=pred_classes.device)


def smooth(y, f=0.05):
    """U/utils/metrics.py:447-452."""
    nf = round(len(y) * f * 2) // 2 + 1
    p = np.ones(nf // 2)
    yp = np.concatenate((p * y[0], y, p * y[-1]), 0)
    return np.convolve(yp, np.ones(nf) / nf, mode="valid")


def compute_ap(recall, precision):
    """U/utils/metrics.py:505-534 (101-point interpolation)."""
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([1.0], precision, [0.0]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    ap = _trapz(np.interp(x, mrec, mpre), x)
    return ap, mpre, mrec


def ap_per_class(tp, conf, pred_cls, target_cls, eps=1e-16):
    """U/utils/metrics.py:537-623 without plotting. Returns (tp, fp, p, r, f1, ap, unique_classes)."""
    i = np.argsort(-conf)
    tp, conf, pred_cls = tp[i], conf[i], pred_cls[i]
    unique_classes, nt = np.unique(target_cls, return_counts=True)
    nc = unique_classes.shape[0]
    x = np.linspace(0, 1, 1000)
    ap, p_curve, r_curve = np.zeros((nc, tp.shape[1])), np.zeros((nc, 1000)), np.zeros((nc, 1000))
    for ci, c in enumerate(unique_classes):
        i = pred_cls == c
        n_l = nt[ci]
        n_p = i.sum()
        if n_p == 0 or n_l == 0:
            continue
        fpc = (1 - tp[i]).cumsum(0)
        tpc = tp[i].cumsum(0)
        recall = tpc / (n_l + eps)
        r_curve[ci] = np.interp(-x, -conf[i], recall[:, 0], left=0)
        precision = tpc / (tpc + fpc)
        p_curve[ci] = np.interp(-x, -conf[i], precision[:, 0], left=1)
        for j in range(tp.shape[1]):
            ap[ci, j], _, _ = compute_ap(recall[:, j], precision[:, j])
    f1_curve = 2 * p_curve * r_curve / (p_curve + r_curve + eps)
    i = smooth(f1_curve.mean(0), 0.1).argmax()
    p, r, f1 = p_curve[:, i], r_curve[:, i], f1_curve[:, i]
    tp = (r * nt).round()
    fp = (tp / (p + eps) - tp).round()
    return tp, fp, p, r, f1, ap, unique_classes.astype(int)


class BoxMetric:
    """U/utils/metrics.py Metric (the scalar summaries)."""

    def __init__(self):
        self.p, self.r, self.f1, self.all_ap, self.ap_class_index = [], [], [], [], []

    def update(self, results):
        self.p, self.r, self.f1, self.all_ap, self.ap_class_index = results

    @property
    def map50(self):
        return float(self.all_ap[:, 0].mean()) if len(self.all_ap) else 0.0

    @property
    def map75(self):
        return float(self.all_ap[:, 5].mean()) if len(self.all_ap) else 0.0

    @property
    def map(self):
        return float(self.all_ap.mean()) if len(self.all_ap) else 0.0

    @property
    def mp(self):
        return float(self.p.mean()) if len(self.p) else 0.0

    @property
    def mr(self):
        return float(self.r.mean()) if len(self.r) else 0.0


class DetMetrics:
    """U/utils/metrics.py:808-896 (keys include mAP75, :866-868)."""

    keys = ["metrics/precision(B)", "metrics/recall(B)", "metrics/mAP50(B)", "metrics/mAP75(B)", "metrics/mAP50-95(B)"]

    def __init__(self, names=None):
        self.names = names or {}
        self.box = BoxMetric()
        self.speed = {}

    def process(self, tp, conf, pred_cls, target_cls):
        res = ap_per_class(tp, conf, pred_cls, target_cls)
        self.box.update((res[2], res[3], res[4], res[5], res[6]))

    @property
    def results_dict(self):
        b = self.box
        return dict(zip(self.keys + ["fitness"], [b.mp, b.mr, b.map50, b.map75, b.map, 0.1 * b.map50 + 0.9 * b.map]))
