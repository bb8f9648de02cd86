"""ndarray frames -> letterboxed fp32 NCHW batch on the GPU, and boxes back to frame coordinates.

BasePredictor.preprocess (U/engine/predictor.py:116-134) for a list of HWC uint8 BGR frames runs
LetterBox (U/data/augment.py:1535-1597) per frame on the CPU with cv2, stacks, flips BGR->RGB,
transposes to NCHW and divides by 255.  Here the host only computes the letterbox geometry (the
reference's own formulas, below) and ships the raw frames to the device once; ydbl_letterbox does
resize + border + channel flip + layout + scaling in one pass straight into the batch the
forward reads.  DetectionPredictor.postprocess (U/models/yolo/detect/predict.py:23-41) maps the
boxes back with scale_boxes (U/utils/ops.py:92-127), done here with device tensor ops.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import _lib


def letterbox_geometry(shape, new_shape=(640, 640), auto=False, scale_fill=False, scaleup=True, center=True,
                       stride=32):
    """LetterBox.__call__ sizes (U/data/augment.py:1560-1588) -> (unpad_h, unpad_w, top, bottom, left, right)."""
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = min(new_shape[0] / shape[0], new_shape[1] / shape[1])
    if not scaleup:  # only scale down
        r = min(r, 1.0)
    uw, uh = int(round(shape[1] * r)), int(round(shape[0] * r))
    dw, dh = new_shape[1] - uw, new_shape[0] - uh
    if auto:  # minimum rectangle
        dw, dh = dw % stride, dh % stride
    elif scale_fill:  # stretch
        dw, dh = 0.0, 0.0
        uw, uh = new_shape[1], new_shape[0]
    if center:
        dw /= 2
        dh /= 2
    top, bottom = int(round(dh - 0.1)) if center else 0, int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)) if center else 0, int(round(dw + 0.1))
    return uh, uw, top, bottom, left, right


def letterbox_batch(frames, imgsz=(640, 640), stride=32, pt=True, device="cuda", pad=114.0, out=None):
    """Frames (list of HWC uint8 BGR ndarrays, or one) -> fp32 [B, 3, H, W] RGB /255 on `device`.

    auto (minimum-rectangle padding) when all frames share a shape, as BasePredictor.pre_transform
    (U/engine/predictor.py:144-158) sets it for PyTorch models.
    """
    if isinstance(frames, np.ndarray) and frames.ndim == 3:
        frames = [frames]
    frames = list(frames)
    if not frames:
        raise ValueError("letterbox_batch: no frames")
    for f in frames:
        if not isinstance(f, np.ndarray) or f.dtype != np.uint8 or f.ndim != 3 or f.shape[2] != 3:
            raise TypeError("frames must be HWC uint8 BGR ndarrays with 3 channels")
        if f.shape[0] < 1 or f.shape[1] < 1:
            raise ValueError("empty frame")
    same = len({f.shape for f in frames}) == 1
    geo = [letterbox_geometry(f.shape[:2], imgsz, auto=same and pt, stride=stride) for f in frames]
    hw = {(g[0] + g[2] + g[3], g[1] + g[4] + g[5]) for g in geo}
    if len(hw) != 1:
        raise ValueError(f"letterboxed frames differ in size {sorted(hw)}; cannot stack")  # np.stack would fail too
    out_h, out_w = hw.pop()
    meta = np.array([[f.shape[0], f.shape[1], g[0], g[1], g[2], g[4]] for f, g in zip(frames, geo)], dtype=np.int32)
    return letterbox_frames(frames, meta, out_h, out_w, device=device, pad=pad, out=out)


def letterbox_frames(frames, meta, out_h, out_w, device="cuda", pad=114.0, out=None):
    """ydbl_letterbox with explicit geometry: meta int32 [b, 6] rows (frame h, frame w, resized h, resized w,
    top, left); each frame is resized (cv2 INTER_LINEAR) to its resized size and placed at (top, left) of an
    out_h x out_w canvas of `pad`.  Returns fp32 [b, 3, out_h, out_w] RGB /255 on `device`."""
    meta = np.ascontiguousarray(meta, dtype=np.int32).reshape(-1, 6)
    b = len(frames)
    if b == 0 or len(meta) != b:
        raise ValueError("letterbox_frames: need one meta row per frame")
    for f, m in zip(frames, meta):
        if tuple(f.shape[:2]) != (m[0], m[1]) or f.dtype != np.uint8 or f.ndim != 3 or f.shape[2] != 3:
            raise ValueError("frame does not match its meta row (HWC uint8 BGR)")
        if m[2] < 1 or m[3] < 1 or m[4] < 0 or m[5] < 0 or m[4] + m[2] > out_h or m[5] + m[3] > out_w:
            raise ValueError(f"resized frame {tuple(m[2:4])} at {tuple(m[4:6])} does not fit {out_h}x{out_w}")
    sizes = [f.size for f in frames]
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    host = torch.empty(int(sum(sizes)), dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for f, o, n in zip(frames, offs, sizes):
        hv[o: o + n] = np.ascontiguousarray(f).reshape(-1)
    dev = torch.device(device)
    src = host.to(dev, non_blocking=True)
    offs_d = torch.from_numpy(offs).to(dev)
    meta_d = torch.from_numpy(meta).to(dev)
    if out is None:
        out = torch.empty((b, 3, out_h, out_w), dtype=torch.float32, device=dev)
    elif out.shape != (b, 3, out_h, out_w) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be contiguous fp32 {(b, 3, out_h, out_w)}")
    d = _lib.LetterboxDesc(src.data_ptr(), offs_d.data_ptr(), meta_d.data_ptr(), b, out_h, out_w, float(pad),
                           out.data_ptr())
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(_lib.lib.ydbl_letterbox(C.byref(d), stream), "ydbl_letterbox")
    # keep the staging buffers alive until the kernel has read them
    torch.cuda.current_stream(dev).synchronize()
    return out


def scale_boxes(img1_shape, boxes: torch.Tensor, img0_shape) -> torch.Tensor:
    """U/utils/ops.py:92-127 (ratio_pad None, padding True, xyxy) + clip_boxes :319-338, in place."""
    gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
    pad = (round((img1_shape[1] - img0_shape[1] * gain) / 2 - 0.1),
           round((img1_shape[0] - img0_shape[0] * gain) / 2 - 0.1))
    boxes[..., 0] -= pad[0]
    boxes[..., 1] -= pad[1]
    boxes[..., 2] -= pad[0]
    boxes[..., 3] -= pad[1]
    boxes[..., :4] /= gain
    boxes[..., 0].clamp_(0, img0_shape[1])
    boxes[..., 1].clamp_(0, img0_shape[0])
    boxes[..., 2].clamp_(0, img0_shape[1])
    boxes[..., 3].clamp_(0, img0_shape[0])
    return boxes
