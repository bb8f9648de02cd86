"""Results / Boxes containers: the `boxes` subset of U/engine/results.py:187-1110.

``Boxes.data`` is ``[n, 6] = x1, y1, x2, y2, conf, cls`` exactly as the
reference builds it in DetectionPredictor.postprocess
(U/models/yolo/detect/predict.py:23-41).  Host-side API of the reference's Results for detection:
indexing, device moves, update (with clip_boxes), verbose, summary, save_txt, to_df / to_csv /
to_json, and plot (boxes + labels drawn with PIL instead of the reference's cv2/PIL Annotator;
same palette, not pixel-identical).
"""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import torch

# U/utils/plotting.py Colors.hexs (the 20-colour detection palette), RGB
_PALETTE = ["042AFF", "0BDBEB", "F3F3F3", "00DFB7", "111F68", "FF6FDD", "FF444F", "CCED00", "00F344", "BD00FF",
            "00B4FF", "DD00BA", "00FFFF", "26C000", "01FFB3", "7D24FF", "7B0068", "FF1B6C", "FC6D2F", "A2FF0B"]


def _color(i: int, bgr: bool = False):
    h = _PALETTE[int(i) % len(_PALETTE)]
    c = tuple(int(h[k:k + 2], 16) for k in (0, 2, 4))
    return c[::-1] if bgr else c


def _clip_boxes(boxes, shape):
    """U/utils/ops.py:319-338."""
    if isinstance(boxes, torch.Tensor):
        boxes[..., 0] = boxes[..., 0].clamp(0, shape[1])
        boxes[..., 1] = boxes[..., 1].clamp(0, shape[0])
        boxes[..., 2] = boxes[..., 2].clamp(0, shape[1])
        boxes[..., 3] = boxes[..., 3].clamp(0, shape[0])
    else:
        boxes[..., [0, 2]] = boxes[..., [0, 2]].clip(0, shape[1])
        boxes[..., [1, 3]] = boxes[..., [1, 3]].clip(0, shape[0])
    return boxes


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

    def __init__(self, orig_img, path, names, boxes=None, speed=None, orig_shape=None):
        """orig_img / boxes may also be zero-argument callables producing them (predict() hands over per-image views
        of its batch buffers that way: built on first access, not for every image of every batch)."""
        self._orig_img = orig_img
        if orig_shape is None and orig_img is not None:
            orig_shape = (orig_img() if callable(orig_img) else orig_img).shape[:2]
        self.orig_shape = tuple(orig_shape) if orig_shape is not None else None
        self.path = path
        self.names = names
        self._boxes_src, self._boxes = boxes, None
        self.speed = speed or {"preprocess": None, "inference": None, "postprocess": None}

    @property
    def orig_img(self):
        if callable(self._orig_img):
            self._orig_img = self._orig_img()
        return self._orig_img

    @orig_img.setter
    def orig_img(self, v):
        self._orig_img = v

    @property
    def boxes(self):
        if self._boxes is None and self._boxes_src is not None:
            src = self._boxes_src() if callable(self._boxes_src) else self._boxes_src
            self._boxes, self._boxes_src = Boxes(src, self.orig_shape), None
        return self._boxes

    @boxes.setter
    def boxes(self, v):
        self._boxes, self._boxes_src = v, None

    def __len__(self):
        return 0 if self.boxes is None else len(self.boxes)

    def __getitem__(self, idx):
        return self._apply("__getitem__", idx)

    def _apply(self, fn, *args, **kwargs):
        r = self.new()
        if self.boxes is not None:
            r.boxes = getattr(self.boxes, fn)(*args, **kwargs)
        return r

    def new(self):
        return Results(self._orig_img, self.path, self.names, None, self.speed, orig_shape=self.orig_shape)

    def update(self, boxes=None):
        """U/engine/results.py:308-334 (boxes): clip to the original image and replace."""
        if boxes is not None:
            self.boxes = Boxes(_clip_boxes(boxes, self.orig_shape), self.orig_shape)

    def cpu(self):
        return self._apply("cpu")

    def numpy(self):
        return self._apply("numpy")

    def cuda(self):
        return self._apply("cuda")

    def to(self, *args, **kwargs):
        return self._apply("to", *args, **kwargs)

    def save_txt(self, txt_file, save_conf=False):
        """U/engine/results.py:665-718 (detection): 'cls xc yc w h [conf]' normalized, appended."""
        texts = []
        if self.boxes is not None and len(self.boxes):
            b = self.boxes.cpu() if isinstance(self.boxes.data, torch.Tensor) else self.boxes
            xywhn = torch.as_tensor(b.xywhn)
            for j in range(len(b)):
                d = b[j]
                c, conf = int(torch.as_tensor(d.cls).item()), float(torch.as_tensor(d.conf).item())
                tid = None if d.id is None else int(torch.as_tensor(d.id).item())
                line = (c, *xywhn[j].view(-1).tolist()) + (conf,) * save_conf + (() if tid is None else (tid,))
                texts.append(("%g " * len(line)).rstrip() % line)
        if texts:
            Path(txt_file).parent.mkdir(parents=True, exist_ok=True)
            with open(txt_file, "a") as f:
                f.writelines(t + "\n" for t in texts)
        return str(txt_file)

    def to_df(self, normalize=False, decimals=5):
        import pandas as pd

        return pd.DataFrame(self.summary(normalize=normalize, decimals=decimals))

    def to_csv(self, normalize=False, decimals=5, *args, **kwargs):
        return self.to_df(normalize=normalize, decimals=decimals).to_csv(*args, **kwargs)

    def to_json(self, normalize=False, decimals=5):
        return json.dumps(self.summary(normalize=normalize, decimals=decimals), indent=2)

    def plot(self, conf=True, line_width=None, labels=True, boxes=True, img=None):
        """Annotated copy of the original image (HWC uint8 BGR ndarray, like the reference's plot())."""
        from PIL import Image, ImageDraw

        im = self.orig_img if img is None else img
        if isinstance(im, torch.Tensor):  # CHW/HWC float 0..1 tensor source -> HWC uint8 BGR
            t = im.detach().float().cpu()
            if t.ndim == 3 and t.shape[0] == 3 and t.shape[-1] != 3:
                t = t.permute(1, 2, 0)
            im = (t.clamp(0, 1) * 255).round().byte().numpy()[..., ::-1]
        im = np.ascontiguousarray(im)
        pil = Image.fromarray(im[..., ::-1].copy())  # BGR -> RGB for PIL
        draw = ImageDraw.Draw(pil)
        lw = line_width or max(round(sum(im.shape[:2]) / 2 * 0.003), 2)
        if boxes and self.boxes is not None:
            data = torch.as_tensor(self.boxes.data).detach().cpu()
            for row in reversed(data.tolist()):
                x1, y1, x2, y2, cf, c = row[0], row[1], row[2], row[3], row[-2], int(row[-1])
                col = _color(c)
                draw.rectangle([x1, y1, x2, y2], outline=col, width=lw)
                if labels:
                    name = self.names[c] if self.names else str(c)
                    text = f"{name} {cf:.2f}" if conf else name
                    tb = draw.textbbox((x1, y1), text)
                    th = tb[3] - tb[1]
                    ty = y1 - th - 2 if y1 - th - 2 >= 0 else y1
                    draw.rectangle([x1, ty, x1 + (tb[2] - tb[0]) + 2, ty + th + 2], fill=col)
                    draw.text((x1 + 1, ty), text, fill=(255, 255, 255))
        return np.ascontiguousarray(np.asarray(pil)[..., ::-1])

    def save(self, filename=None, **kwargs):
        from PIL import Image

        filename = filename or f"results_{Path(self.path).name}"
        Image.fromarray(self.plot(**kwargs)[..., ::-1].copy()).save(filename)
        return filename

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
        """U/engine/results.py:630-663 (detection)."""
        if self.boxes is None or len(self.boxes) == 0:
            return "(no detections), "
        cls = self.boxes.cls.int().tolist() if isinstance(self.boxes.cls, torch.Tensor) else list(self.boxes.cls)
        s = ""
        for c in sorted(set(cls)):
            n = cls.count(c)
            s += f"{n} {self.names[int(c)]}{'s' * (n > 1)}, "
        return s
