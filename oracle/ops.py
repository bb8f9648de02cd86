"""Oracle restatement of box ops and NMS (TEST INFRASTRUCTURE ONLY).

Follows ``U/utils/ops.py:167-338, 416-433, 850-854`` and restates
``torchvision.ops.nms`` (torchvision 0.23.0, CPU kernel, not vendored in the
reference): stable descending score sort, greedy sweep, suppress j when
``inter / (area_i + area_j - inter) > iou_threshold`` evaluated as
float-IoU compared against a double threshold, areas without +1.
"""

from __future__ import annotations

import numpy as np
import torch


def xywh2xyxy(x):
    """utils/ops.py:416-433 (fp32 result via empty_like :850-854)."""
    y = torch.empty_like(x, dtype=torch.float32)
    xy = x[..., :2]
    wh = x[..., 2:] / 2
    y[..., :2] = xy - wh
    y[..., 2:] = xy + wh
    return y


def clip_boxes(boxes, shape):
    """utils/ops.py:319-338 (tensor branch)."""
    boxes[..., 0] = boxes[..., 0].clamp(0, shape[1])
    boxes[..., 1] = boxes[..., 1].clamp(0, shape[0])
    boxes[..., 2] = boxes[..., 2].clamp(0, shape[1])
    boxes[..., 3] = boxes[..., 3].clamp(0, shape[0])
    return boxes


def nms_torchvision(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float) -> torch.Tensor:
    """Greedy NMS with torchvision's CPU-kernel semantics; returns int64 keep indices in score order.

    Vectorised per kept box; the float32 arithmetic per (i, j) pair is the
    kernel's: xx1=max, yy1=max, xx2=min, yy2=min, w=max(0,xx2-xx1),
    h=max(0,yy2-yy1), inter=w*h, ovr=inter/(area_i+area_j-inter).
    """
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.int64)
    lib = _c_nms()
    if lib is not None and not _FORCE_PY_NMS:
        b = np.ascontiguousarray(boxes.detach().to(torch.float32).cpu().numpy())
        s = np.ascontiguousarray(scores.detach().to(torch.float32).cpu().numpy())
        keep = np.empty(n, dtype=np.int64)
        k = lib.ydbl_oracle_nms(b.ctypes.data, s.ctypes.data, n, float(iou_threshold), keep.ctypes.data)
        if k < 0:
            raise MemoryError("ydbl_oracle_nms")
        return torch.from_numpy(keep[:k].copy())
    return nms_torchvision_py(boxes, scores, iou_threshold)


_FORCE_PY_NMS = False
_C_NMS = []


def _c_nms():
    """oracle/_nms.so (oracle/nms.c, the same kernel in C, built by `make -C oracle`) when present."""
    if not _C_NMS:
        import ctypes
        from pathlib import Path

        so = Path(__file__).resolve().parent / "_nms.so"
        lib = None
        if so.exists():
            lib = ctypes.CDLL(str(so))
            lib.ydbl_oracle_nms.restype = ctypes.c_int64
            lib.ydbl_oracle_nms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double,
                                            ctypes.c_void_p]
        _C_NMS.append(lib)
    return _C_NMS[0]


def nms_torchvision_py(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float) -> torch.Tensor:
    """nms_torchvision in numpy (the restatement oracle/nms.c is checked against, tests/test_oracle.py)."""
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.int64)
    b = boxes.detach().to(torch.float32).cpu().numpy()
    s = scores.detach().to(torch.float32).cpu().numpy()
    order = np.argsort(-s, kind="stable")  # stable descending (ties keep input order)
    x1, y1, x2, y2 = (b[order, k].astype(np.float32) for k in range(4))
    areas = ((x2 - x1) * (y2 - y1)).astype(np.float32)
    suppressed = np.zeros(n, dtype=bool)
    keep = []
    thr = np.float64(iou_threshold)
    for i in range(n):
        if suppressed[i]:
            continue
        keep.append(order[i])
        j = slice(i + 1, n)
        xx1 = np.maximum(x1[i], x1[j])
        yy1 = np.maximum(y1[i], y1[j])
        xx2 = np.minimum(x2[i], x2[j])
        yy2 = np.minimum(y2[i], y2[j])
        w = np.maximum(np.float32(0), xx2 - xx1)
        h = np.maximum(np.float32(0), yy2 - yy1)
        inter = (w * h).astype(np.float32)
        with np.errstate(invalid="ignore", divide="ignore"):
            ovr = (inter / ((areas[i] + areas[j]) - inter)).astype(np.float32)
        suppressed[j] |= ovr.astype(np.float64) > thr
    return torch.as_tensor(np.asarray(keep, dtype=np.int64))


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, max_det=300, nc=0, max_nms=30000, max_wh=7680):
    """utils/ops.py:167-316 restated (no labels, no masks, not rotated, no time limit truncation)."""
    if isinstance(prediction, (list, tuple)):
        prediction = prediction[0]
    bs = prediction.shape[0]
    nc = nc or (prediction.shape[1] - 4)
    mi = 4 + nc
    xc = prediction[:, 4:mi].amax(1) > conf_thres
    multi_label &= nc > 1
    prediction = prediction.transpose(-1, -2).clone()
    prediction[..., :4] = xywh2xyxy(prediction[..., :4])
    if classes is not None:
        classes = torch.tensor(classes)
    output = [torch.zeros((0, 6))] * bs
    for xi, x in enumerate(prediction):
        x = x[xc[xi]]
        if not x.shape[0]:
            continue
        box, cls = x[:, :4], x[:, 4:mi]
        if multi_label:
            i, j = torch.where(cls > conf_thres)
            x = torch.cat((box[i], x[i, 4 + j, None], j[:, None].float()), 1)
        else:
            conf, j = cls.max(1, keepdim=True)
            x = torch.cat((box, conf, j.float()), 1)[conf.view(-1) > conf_thres]
        if classes is not None:
            x = x[(x[:, 5:6] == classes).any(1)]
        n = x.shape[0]
        if not n:
            continue
        if n > max_nms:
            # the reference calls a non-stable argsort (U/utils/ops.py:286): the order of equal scores is
            # unspecified there; the restatement (and the GPU kernel) fix it to the stable order
            x = x[x[:, 4].argsort(descending=True, stable=True)[:max_nms]]
        c = x[:, 5:6] * (0 if agnostic else max_wh)
        keep = nms_torchvision(x[:, :4] + c, x[:, 4], iou_thres)[:max_det]
        output[xi] = x[keep]
    return output
