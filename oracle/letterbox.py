"""Oracle restatement of the predictor's ndarray preprocessing (TEST INFRASTRUCTURE ONLY).

LetterBox.__call__ (U/data/augment.py:1535-1597) with cv2.resize INTER_LINEAR and
cv2.copyMakeBorder(114), then BasePredictor.preprocess (U/engine/predictor.py:116-134):
BGR->RGB, HWC->CHW, float, /255.  cv2 (opencv-python >= 4.6 per the reference's requirements) is
not vendored and not installed here, so its uint8 INTER_LINEAR is restated from OpenCV 4.x
imgproc/src/resize.cpp (generic fixed-point path, the 2x INTER_AREA shortcut, 128-bit SIMD
vertical pass VResizeLinearVec_32s8u plus scalar tail).  PARITY UNPINNED against real cv2: no
fixture of the reference holds a resized frame; the device kernel is checked bit-exact against this
restatement and the geometry (sizes, padding) against the reference's formulas.
"""

from __future__ import annotations

import numpy as np


def letterbox_geometry(shape, new_shape=(640, 640), auto=False, scale_fill=False, scaleup=True, center=True,
                       stride=32):
    """augment.py:1560-1588 -> (unpad_h, unpad_w, top, bottom, left, right)."""
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = min(new_shape[0] / shape[0], new_shape[1] / shape[1])
    if not scaleup:
        r = min(r, 1.0)
    new_unpad = int(round(shape[1] * r)), int(round(shape[0] * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:
        dw, dh = np.mod(dw, stride), np.mod(dh, stride)
    elif scale_fill:
        dw, dh = 0.0, 0.0
        new_unpad = (new_shape[1], new_shape[0])
    if center:
        dw /= 2
        dh /= 2
    top, bottom = int(round(dh - 0.1)) if center else 0, int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)) if center else 0, int(round(dw + 0.1))
    return new_unpad[1], new_unpad[0], top, bottom, left, right


def _taps(dst: int, src: int, clamp_coef: bool):
    inv = dst / src
    scale = 1.0 / inv
    f = ((np.arange(dst) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if clamp_coef:  # columns: sx<0 -> (0, fx=0); sx>=src-1 -> (src-1, fx=0)
        lo = s < 0
        f[lo], s[lo] = 0, 0
        hi = s >= src - 1
        f[hi], s[hi] = 0, src - 1
    a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048)).astype(np.int64)
    return s, a0, a1


def resize_linear_u8(img: np.ndarray, dh: int, dw: int) -> np.ndarray:
    """cv2.resize(img, (dw, dh), interpolation=INTER_LINEAR) for HWC uint8, OpenCV 4.x semantics."""
    sh, sw, cn = img.shape
    S = img.astype(np.int64)
    if sw == 2 * dw and sh == 2 * dh:  # is_area_fast with iscale 2 -> INTER_AREA fast
        return ((S[0::2, 0::2] + S[0::2, 1::2] + S[1::2, 0::2] + S[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    sx, a0, a1 = _taps(dw, sw, True)
    a1 = np.where(sx + 1 >= sw, 0, a1)
    sx1 = np.minimum(sx + 1, sw - 1)
    hx = S[:, sx, :] * a0[None, :, None] + S[:, sx1, :] * a1[None, :, None]  # [sh, dw, cn] int32-exact
    sy, b0, b1 = _taps(dh, sh, False)
    r0 = hx[np.clip(sy, 0, sh - 1)]
    r1 = hx[np.clip(sy + 1, 0, sh - 1)]
    b0, b1 = b0[:, None, None], b1[:, None, None]
    scalar = (r0 * b0 + r1 * b1 + (1 << 21)) >> 22
    simd = ((((r0 >> 4) * b0) >> 16) + (((r1 >> 4) * b1) >> 16) + 2) >> 2
    width = dw * cn
    end = (width // 16) * 16
    while end < width - 8:
        end += 8
    e = (np.arange(dw)[:, None] * cn + np.arange(cn)[None, :])[None]
    out = np.where(e < end, simd, scalar)
    return np.clip(out, 0, 255).astype(np.uint8)


def letterbox(img: np.ndarray, new_shape=(640, 640), auto=False, stride=32, pad=114) -> np.ndarray:
    """LetterBox(new_shape, auto, stride)(image=img): HWC uint8 BGR canvas."""
    uh, uw, top, bottom, left, right = letterbox_geometry(img.shape[:2], new_shape, auto=auto, stride=stride)
    if img.shape[:2] != (uh, uw):
        img = resize_linear_u8(img, uh, uw)
    out = np.full((uh + top + bottom, uw + left + right, img.shape[2]), pad, dtype=np.uint8)
    out[top: top + uh, left: left + uw] = img
    return out


def preprocess(frames, imgsz=(640, 640), stride=32, pt=True) -> np.ndarray:
    """BasePredictor.preprocess for a list of HWC uint8 BGR frames -> fp32 NCHW RGB /255."""
    same_shapes = len({x.shape for x in frames}) == 1
    im = np.stack([letterbox(x, imgsz, auto=same_shapes and pt, stride=stride) for x in frames])
    im = np.ascontiguousarray(im[..., ::-1].transpose((0, 3, 1, 2)))
    return im.astype(np.float32) / np.float32(255)
