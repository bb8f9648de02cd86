"""Results / Boxes containers: the `boxes` subset of U/engine/results.py:187-1110.

``Boxes.data`` is ``[n, 6] = x1, y1, x2, y2, conf, cls`` exactly as the
reference builds it in DetectionPredictor.postprocess
(U/models/yolo/detect/predict.py:23-41).
"""

from __future__ import annotations

import numpy as np
import torch


class Boxes:
    """U/engine/results.py:938-1110 (detection subset)."""

    def __init__(self, boxes, orig_shape):
        if boxes.ndim == 1:
            boxes = boxes[None, :]
        n = boxes.shape[-1]
        assert n in {6, 7}, f"expected 6 or 7 values but got {n}"
        self.data = boxes
        self.orig_shape = tuple(orig_shape)
        self.is_track = n == 7

    def _new(self, data):
        return Boxes(data, self.orig_shape)

    def cpu(self):
        return self._new(self.data.cpu()) if isinstance(self.data, torch.Tensor) else self

    def numpy(self):
        return self._new(self.data.cpu().numpy() if isinstance(self.data, torch.Tensor) else self.data)

    def cuda(self):
        return self._new(torch.as_tensor(self.data).cuda())

    def to(self, *args, **kwargs):
        return self._new(torch.as_tensor(self.data).to(*args, **kwargs))

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self._new(self.data[idx])

    @property
    def shape(self):
        return self.data.shape

    @property
    def xyxy(self):
        return self.data[:, :4]

    @property
    def conf(self):
        return self.data[:, -2]

    @property
    def cls(self):
        return self.data[:, -1]

    @property
    def id(self):
        return self.data[:, -3] if self.is_track else None

    @property
    def xywh(self):
        x = self.xyxy
        y = torch.empty_like(x) if isinstance(x, torch.Tensor) else np.empty_like(x)
        y[..., 0] = (x[..., 0] + x[..., 2]) / 2
        y[..., 1] = (x[..., 1] + x[..., 3]) / 2
        y[..., 2] = x[..., 2] - x[..., 0]
        y[..., 3] = x[..., 3] - x[..., 1]
        return y

    @property
    def xyxyn(self):
        x = self.xyxy.clone() if isinstance(self.xyxy, torch.Tensor) else np.copy(self.xyxy)
        x[..., [0, 2]] /= self.orig_shape[1]
        x[..., [1, 3]] /= self.orig_shape[0]
        return x

    @property
    def xywhn(self):
        x = self.xywh
        x[..., [0, 2]] /= self.orig_shape[1]
        x[..., [1, 3]] /= self.orig_shape[0]
        return x


class Results:
    """U/engine/results.py:187- (detection subset: boxes, names, orig_shape, speed)."""

    def __init__(self, orig_img, path, names, boxes=None, speed=None):
        self.orig_img = orig_img
        self.orig_shape = tuple(orig_img.shape[:2]) if orig_img is not None else None
        self.path = path
        self.names = names
        self.boxes = Boxes(boxes, self.orig_shape) if boxes is not None else None
        self.speed = speed or {"preprocess": None, "inference": None, "postprocess": None}

    def __len__(self):
        return 0 if self.boxes is None else len(self.boxes)

    def cpu(self):
        r = Results(self.orig_img, self.path, self.names, None, self.speed)
        r.boxes = self.boxes.cpu() if self.boxes is not None else None
        return r

    def numpy(self):
        r = Results(self.orig_img, self.path, self.names, None, self.speed)
        r.boxes = self.boxes.numpy() if self.boxes is not None else None
        return r

    def summary(self, normalize=False, decimals=5):
        out = []
        if self.boxes is None:
            return out
        h, w = self.orig_shape
        for row in self.boxes.data.tolist():
            x1, y1, x2, y2, conf, cls = row[:6]
            if normalize:
                x1, x2, y1, y2 = x1 / w, x2 / w, y1 / h, y2 / h
            out.append({"name": self.names[int(cls)], "class": int(cls), "confidence": round(conf, decimals),
                        "box": {k: round(v, decimals) for k, v in zip(("x1", "y1", "x2", "y2"), (x1, y1, x2, y2))}})
        return out

    def verbose(self):
        if self.boxes is None or len(self.boxes) == 0:
            return "(no detections), "
        cls = self.boxes.cls.int().tolist() if isinstance(self.boxes.cls, torch.Tensor) else list(self.boxes.cls)
        s = ""
        for c in sorted(set(cls)):
            n = cls.count(c)
            s += f"{n} {self.names[int(c)]}{'s' * (n > 1)}, "
        return s
