"""Detection metrics for the mAP acceptance check (host numpy, as the reference computes them).

Restates U/utils/metrics.py:447-452 (smooth), :505-534 (compute_ap, 101-point COCO interpolation),
:537-623 (ap_per_class) and :808-896 (DetMetrics keys incl. mAP75).  The per-image TP matrix
(box_iou + match_predictions) runs on the device: ydbl_match_predictions, see engine/validator.py;
its host restatement is the checker in oracle/metrics.py.
"""

from __future__ import annotations

import numpy as np
import torch

IOUV = torch.linspace(0.5, 0.95, 10)  # U/models/yolo/detect/val.py:36 (iou vector for mAP@0.5:0.95)

_trapz = getattr(np, "trapezoid", None) or np.trapz


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
