"""Box utilities and HIP-backed NMS with the reference signature (U/utils/ops.py)."""

from __future__ import annotations

import math

import torch

from .. import _lib
from .._lib import NmsDesc, PredCandDesc


def make_divisible(x, divisor):
    """U/utils/ops.py:130-143."""
    if isinstance(divisor, torch.Tensor):
        divisor = int(divisor.max())
    return math.ceil(x / divisor) * divisor


def xywh2xyxy(x):
    """U/utils/ops.py:416-433."""
    assert x.shape[-1] == 4, f"input shape last dimension expected 4 but input shape is {x.shape}"
    y = torch.empty_like(x, dtype=torch.float32)
    xy = x[..., :2]
    wh = x[..., 2:] / 2
    y[..., :2] = xy - wh
    y[..., 2:] = xy + wh
    return y


def clip_boxes(boxes, shape):
    """U/utils/ops.py:319-338."""
    boxes[..., 0] = boxes[..., 0].clamp(0, shape[1])
    boxes[..., 1] = boxes[..., 1].clamp(0, shape[0])
    boxes[..., 2] = boxes[..., 2].clamp(0, shape[1])
    boxes[..., 3] = boxes[..., 3].clamp(0, shape[0])
    return boxes


def scale_boxes(img1_shape, boxes, img0_shape, ratio_pad=None, padding=True, xywh=False):
    """U/utils/ops.py:92-127."""
    if ratio_pad is None:
        gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
        pad = (round((img1_shape[1] - img0_shape[1] * gain) / 2 - 0.1),
               round((img1_shape[0] - img0_shape[0] * gain) / 2 - 0.1))
    else:
        gain = ratio_pad[0][0]
        pad = ratio_pad[1]
    if padding:
        boxes[..., 0] -= pad[0]
        boxes[..., 1] -= pad[1]
        if not xywh:
            boxes[..., 2] -= pad[0]
            boxes[..., 3] -= pad[1]
    boxes[..., :4] /= gain
    return clip_boxes(boxes, img0_shape)


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, labels=(), max_det=300, nc=0, max_time_img=0.05, max_nms=30000,
                        max_wh=7680, in_place=True, rotated=False):
    """U/utils/ops.py:167-316 on the GPU: ydbl_pred_candidates + ydbl_nms.

    prediction: CUDA tensor [B, 4+nc, A] (xywh pixels, class scores), or a (pred, feats) tuple.
    Returns a list of [n_i, 6] CUDA tensors (x1, y1, x2, y2, conf, cls).  The reference's NMS time
    limit (max_time_img) never truncates here; masks, apriori labels and rotated boxes are not on
    the DBL path and raise.  The prediction tensor is not modified (in_place has no effect).
    """
    assert 0 <= conf_thres <= 1, f"Invalid Confidence threshold {conf_thres}, valid values are between 0.0 and 1.0"
    assert 0 <= iou_thres <= 1, f"Invalid IoU {iou_thres}, valid values are between 0.0 and 1.0"
    if isinstance(prediction, (list, tuple)):
        prediction = prediction[0]
    if rotated or (labels is not None and len(labels)):
        raise NotImplementedError("rotated / autolabel NMS is not on the YOLO-DBL path")
    if not prediction.is_cuda:
        raise RuntimeError("ydbl non_max_suppression runs on the GPU only (prediction must be a CUDA tensor)")
    bs = prediction.shape[0]
    nc = nc or (prediction.shape[1] - 4)
    if prediction.shape[1] != 4 + nc:
        raise NotImplementedError("mask channels are not on the YOLO-DBL path")
    A = prediction.shape[2]
    multi_label = bool(multi_label) and nc > 1
    pred = prediction.detach().float().contiguous()
    dev = pred.device
    cap = A * nc if multi_label else A
    cand_box = torch.empty((bs, cap, 4), dtype=torch.float32, device=dev)
    cand_score = torch.empty((bs, cap), dtype=torch.float32, device=dev)
    cand_cls = torch.empty((bs, cap), dtype=torch.int32, device=dev)
    cand_idx = torch.empty((bs, cap), dtype=torch.int32, device=dev)
    cand_count = torch.empty((bs,), dtype=torch.int32, device=dev)
    cls_t = torch.tensor(list(classes), dtype=torch.int32, device=dev) if classes is not None else None
    stream = torch.cuda.current_stream(dev).cuda_stream
    pd = PredCandDesc(pred.data_ptr(), bs, nc, A, float(conf_thres), int(multi_label),
                      cls_t.data_ptr() if cls_t is not None else None, len(cls_t) if cls_t is not None else 0,
                      cand_box.data_ptr(), cand_score.data_ptr(), cand_cls.data_ptr(), cand_idx.data_ptr(),
                      cand_count.data_ptr(), cap)
    _lib.check(_lib.lib.ydbl_pred_candidates(pd, stream), "ydbl_pred_candidates")
    out = torch.zeros((bs, max_det, 6), dtype=torch.float32, device=dev)
    cnt = torch.zeros((bs,), dtype=torch.int32, device=dev)
    ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(bs, cap, max_nms)), dtype=torch.uint8, device=dev)  # zero-filled once (include/ydbl.h)
    nd = NmsDesc(cand_box.data_ptr(), cand_score.data_ptr(), cand_cls.data_ptr(), cand_idx.data_ptr(),
                 cand_count.data_ptr(), bs, cap, float(iou_thres), int(max_det), int(max_nms), int(bool(agnostic)),
                 float(max_wh), 0.0, 0.0, out.data_ptr(), cnt.data_ptr(), ws.data_ptr())
    _lib.check(_lib.lib.ydbl_nms(nd, stream), "ydbl_nms")
    counts = cnt.tolist()
    return [out[i, : counts[i]] for i in range(bs)]
