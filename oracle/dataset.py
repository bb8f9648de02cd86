"""Oracle restatement of the reference's val-split data pipeline and validation loop (TEST INFRASTRUCTURE ONLY).

Follows, step by step and per image as the reference runs them:
- check_det_dataset (U/data/utils.py:301-391): YAML keys, names/nc, path resolution (relative 'path' taken from
  the YAML's folder; the reference's settings datasets_dir does not exist here);
- get_img_files (U/data/base.py:106-130), img2label_paths (U/data/utils.py:44-47), verify_image_label (:97-165);
- set_rectangle (U/data/base.py:261-284);
- load_image (U/data/base.py:151-187) with cv2.resize INTER_LINEAR (restated in oracle/letterbox.py);
- LetterBox(new_shape=rect_shape, scaleup=False) + _update_labels (U/data/augment.py:1535-1630);
- Format(bbox_format='xywh', normalize=True) (:2011-2076), collate_fn (U/data/dataset.py:232-248);
- DetectionValidator.preprocess/_prepare_batch/_prepare_pred/update_metrics (U/models/yolo/detect/val.py:50-172)
  with scale_boxes(ratio_pad) (U/utils/ops.py:92-127).
Images are decoded with PIL into cv2.imread's BGR layout (cv2 is not installed: parity of the decode is unpinned
for JPEG; PNG is lossless).
"""

from __future__ import annotations

import math
import os
from pathlib import Path

import numpy as np
import torch

from oracle.letterbox import resize_linear_u8
from oracle.metrics import box_iou, match_predictions
from oracle.ops import clip_boxes, non_max_suppression, xywh2xyxy

IMG_FORMATS = {"bmp", "dng", "jpeg", "jpg", "mpo", "png", "tif", "tiff", "webp", "pfm", "heic"}


def data_yaml(file) -> dict:
    import yaml

    file = Path(file)
    data = yaml.safe_load(file.read_text())
    if "val" not in data and "validation" in data:
        data["val"] = data.pop("validation")
    names = data.get("names") or [f"class_{i}" for i in range(data["nc"])]
    data["nc"] = len(names)
    root = Path(data.get("path") or file.parent)
    root = root if root.is_absolute() else (file.parent / root).resolve()
    v = data["val"]
    data["val"] = [str((root / x).resolve()) for x in v] if isinstance(v, list) else str((root / v).resolve())
    return data


def image_files(img_path):
    out = []
    for p in img_path if isinstance(img_path, list) else [img_path]:
        p = Path(p)
        if p.is_dir():
            out += [str(q) for q in p.rglob("*.*")]
        else:
            lines = p.read_text().strip().splitlines()
            out += [str(p.parent) + os.sep + x[2:] if x.startswith("./") else x for x in lines]
    return sorted(x for x in out if x.split(".")[-1].lower() in IMG_FORMATS)


def label_file(im_file):
    a, b = f"{os.sep}images{os.sep}", f"{os.sep}labels{os.sep}"
    head, sep, tail = im_file.rpartition(a)
    p = head + b + tail if sep else im_file
    return p.rsplit(".", 1)[0] + ".txt"


def read_labels(im_file, num_cls):
    """verify_image_label -> (hw, lb [n, 5]) or None when the pair is corrupt."""
    from PIL import Image

    try:
        im = Image.open(im_file)
        im.verify()
        w, h = im.size
        if im.format == "JPEG":
            rot = im.getexif().get(274, None)
            if rot in (6, 8):
                w, h = h, w
        if h <= 9 or w <= 9 or im.format.lower() not in IMG_FORMATS:
            return None
        lf = label_file(im_file)
        lb = np.zeros((0, 5), np.float32)
        if os.path.isfile(lf):
            rows = [r.split() for r in open(lf).read().strip().splitlines() if r]
            if any(len(r) > 6 for r in rows):
                cls = np.array([r[0] for r in rows], np.float32)
                boxes = []
                for r in rows:
                    pts = np.array(r[1:], np.float32).reshape(-1, 2)
                    x1, y1, x2, y2 = pts[:, 0].min(), pts[:, 1].min(), pts[:, 0].max(), pts[:, 1].max()
                    boxes.append([(x1 + x2) / 2, (y1 + y2) / 2, x2 - x1, y2 - y1])
                rows = np.concatenate([cls[:, None], np.array(boxes)], 1)
            if len(rows):
                lb = np.array(rows, np.float32)
                if lb.shape[1] != 5 or lb[:, 1:].max() > 1 or lb.min() < 0 or lb[:, 0].max() > num_cls:
                    return None
                _, i = np.unique(lb, axis=0, return_index=True)
                if len(i) < len(lb):
                    lb = lb[i]
        return (h, w), lb
    except Exception:  # noqa: BLE001
        return None


def imread_bgr(f):
    from PIL import Image, ImageOps

    im = Image.open(f)
    if im.format == "JPEG":
        im = ImageOps.exif_transpose(im)
    return np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])


class ValData:
    """YOLODataset(augment=False, rect, pad=0.5) restated; ``batch(i)`` = the collated batch i."""

    def __init__(self, img_path, imgsz, batch_size, stride=32, num_cls=80, rect=True):
        self.imgsz, self.bs, self.stride, self.rect = imgsz, batch_size, stride, rect
        self.items = []
        for f in image_files(img_path):
            r = read_labels(f, num_cls)
            if r is not None:
                self.items.append({"im_file": f, "shape": r[0], "lb": r[1]})
        n = len(self.items)
        self.bi = np.floor(np.arange(n) / batch_size).astype(int)
        if rect:
            s = np.array([it["shape"] for it in self.items])
            ar = s[:, 0] / s[:, 1]
            order = ar.argsort()
            self.items = [self.items[i] for i in order]
            ar = ar[order]
            shapes = []
            for i in range(self.bi[-1] + 1):
                a = ar[self.bi == i]
                shapes.append([a.max(), 1] if a.max() < 1 else ([1, 1 / a.min()] if a.min() > 1 else [1, 1]))
            self.batch_shapes = np.ceil(np.array(shapes) * imgsz / stride + 0.5).astype(int) * stride

    def __len__(self):
        return int(self.bi[-1]) + 1 if len(self.items) else 0

    def sample(self, i):
        it = self.items[i]
        im = imread_bgr(it["im_file"])
        h0, w0 = im.shape[:2]
        r = self.imgsz / max(h0, w0)
        if r != 1:
            w, h = min(math.ceil(w0 * r), self.imgsz), min(math.ceil(h0 * r), self.imgsz)
            im = resize_linear_u8(im, h, w)
        h, w = im.shape[:2]
        # LetterBox(scaleup=False) with the rect shape
        new_shape = tuple(self.batch_shapes[self.bi[i]]) if self.rect else (self.imgsz, self.imgsz)
        rr = min(min(new_shape[0] / h, new_shape[1] / w), 1.0)
        uw, uh = int(round(w * rr)), int(round(h * rr))
        dw, dh = (new_shape[1] - uw) / 2, (new_shape[0] - uh) / 2
        img = im if (w, h) == (uw, uh) else resize_linear_u8(im, uh, uw)
        top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
        left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
        canvas = np.full((uh + top + bottom, uw + left + right, 3), 114, np.uint8)
        canvas[top: top + uh, left: left + uw] = img
        # Instances: xywh normalized -> xyxy, denormalize by the load_image size, scale(rr), add_padding
        b = it["lb"][:, 1:].copy()
        xy, wh = b[:, :2], b[:, 2:] / 2
        b = np.concatenate([xy - wh, xy + wh], 1).astype(np.float32)
        for k, s in enumerate((w, h, w, h)):
            b[:, k] *= s
        for k in range(4):
            b[:, k] *= rr
        for k, s in enumerate((left, top, left, top)):
            b[:, k] += s
        # Format: xyxy -> xywh, torch, normalized by the letterboxed size
        H, W = canvas.shape[:2]
        xywh = np.empty_like(b)
        xywh[:, 0], xywh[:, 1] = (b[:, 0] + b[:, 2]) / 2, (b[:, 1] + b[:, 3]) / 2
        xywh[:, 2], xywh[:, 3] = b[:, 2] - b[:, 0], b[:, 3] - b[:, 1]
        bt = torch.from_numpy(xywh) if len(b) else torch.zeros((0, 4))
        bt[:, [0, 2]] /= W
        bt[:, [1, 3]] /= H
        img_t = torch.from_numpy(np.ascontiguousarray(canvas.transpose(2, 0, 1)[::-1]))  # BGR->RGB CHW uint8
        return {"img": img_t, "cls": torch.from_numpy(it["lb"][:, 0:1].copy()), "bboxes": bt,
                "ori_shape": (h0, w0), "ratio_pad": ((h / h0, w / w0), (left, top)), "im_file": it["im_file"]}

    def batch(self, k):
        idx = [i for i in range(len(self.items)) if self.bi[i] == k]
        ss = [self.sample(i) for i in idx]
        return {"img": torch.stack([s["img"] for s in ss]), "cls": torch.cat([s["cls"] for s in ss]),
                "bboxes": torch.cat([s["bboxes"] for s in ss]),
                "batch_idx": torch.cat([torch.full((len(s["cls"]),), j, dtype=torch.float32) for j, s in enumerate(ss)]),
                "ori_shape": [s["ori_shape"] for s in ss], "ratio_pad": [s["ratio_pad"] for s in ss],
                "im_file": [s["im_file"] for s in ss]}


def scale_boxes_ratio_pad(boxes, img0_shape, ratio_pad):
    gain, pad = ratio_pad[0][0], ratio_pad[1]
    boxes[..., 0] -= pad[0]
    boxes[..., 1] -= pad[1]
    boxes[..., 2] -= pad[0]
    boxes[..., 3] -= pad[1]
    boxes[..., :4] /= gain
    return clip_boxes(boxes, img0_shape)


@torch.inference_mode()
def validate(model, data: ValData, conf=0.001, iou=0.7, max_det=300):
    """BaseValidator loop on the CPU with the oracle model -> stats dict of numpy arrays (tp, conf, pred_cls,
    target_cls) in the reference's image order, plus the letterboxed input batches."""
    stats = {"tp": [], "conf": [], "pred_cls": [], "target_cls": []}
    batches = []
    iouv = torch.linspace(0.5, 0.95, 10)
    for k in range(len(data)):
        bt = data.batch(k)
        batches.append(bt["img"])
        x = bt["img"].float() / 255
        y, _ = model(x)
        preds = non_max_suppression(y, conf, iou, multi_label=True, max_det=max_det)
        H, W = x.shape[2:]
        for si, pred in enumerate(preds):
            idx = bt["batch_idx"] == si
            cls = bt["cls"][idx].squeeze(-1)
            bbox = bt["bboxes"][idx]
            if len(cls):
                bbox = xywh2xyxy(bbox) * torch.tensor((H, W))[[1, 0, 1, 0]]
                scale_boxes_ratio_pad(bbox, bt["ori_shape"][si], bt["ratio_pad"][si])
            if len(pred) == 0:
                if len(cls):
                    stats["tp"].append(torch.zeros(0, 10, dtype=torch.bool))
                    stats["conf"].append(torch.zeros(0))
                    stats["pred_cls"].append(torch.zeros(0))
                    stats["target_cls"].append(cls)
                continue
            predn = pred.clone()
            scale_boxes_ratio_pad(predn[:, :4], bt["ori_shape"][si], bt["ratio_pad"][si])
            tp = torch.zeros(len(pred), 10, dtype=torch.bool)
            if len(cls):
                tp = match_predictions(predn[:, 5], cls, box_iou(bbox, predn[:, :4]), iouv)
            stats["tp"].append(tp)
            stats["conf"].append(predn[:, 4])
            stats["pred_cls"].append(predn[:, 5])
            stats["target_cls"].append(cls)
    return {k: torch.cat(v).numpy() for k, v in stats.items()}, batches
