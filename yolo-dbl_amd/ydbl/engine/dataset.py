"""YOLO-format detection datasets for ``.val(data=...)``: the host side of the val input pipeline.

Restates the val split of the reference's data stack (no augmentation, no label/image cache files):
- check_det_dataset (U/data/utils.py:301-391) and find_dataset_yaml (:279-298): data YAML -> dict with
  resolved 'val' path(s), 'names', 'nc';
- BaseDataset.get_img_files (U/data/base.py:106-130), img2label_paths (U/data/utils.py:44-47) and
  verify_image_label (:97-165) through YOLODataset.get_labels/cache_labels (U/data/dataset.py:66-172);
- set_rectangle (U/data/base.py:261-284): images sorted by aspect ratio, one padded shape per batch;
- load_image (U/data/base.py:151-187) + LetterBox(scaleup=False) with the batch's rect shape
  (U/data/augment.py:1535-1601) + Format(xywh, normalize) (:2011-2076) + collate_fn (U/data/dataset.py:232-248).

Images are decoded on the host (PIL; cv2 is not part of this image: cv2.imread's BGR layout and EXIF rotation
are restated) and shipped to the GPU as raw uint8.  The long-side resize of load_image (cv2 INTER_LINEAR) and the
LetterBox border are one ydbl_letterbox launch per batch: with scaleup=False LetterBox never resizes an image
that load_image already fit inside its rect shape (checked per image below), so resize-then-pad is one pass.
"""

from __future__ import annotations

import glob
import math
import os
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

IMG_FORMATS = {"bmp", "dng", "jpeg", "jpg", "mpo", "png", "tif", "tiff", "webp", "pfm", "heic"}  # U/data/utils.py:38


# ----------------------------------------------------------------------------------------------- data YAML
def find_dataset_yaml(path: Path) -> Path:
    """U/data/utils.py:279-298."""
    files = list(path.glob("*.yaml")) or list(path.rglob("*.yaml"))
    if not files:
        raise FileNotFoundError(f"no YAML file found in '{path.resolve()}'")
    if len(files) > 1:
        files = [f for f in files if f.stem == path.stem]
    if len(files) != 1:
        raise FileNotFoundError(f"expected 1 YAML file in '{path.resolve()}', but found {len(files)}")
    return files[0]


def check_det_dataset(dataset) -> dict:
    """U/data/utils.py:301-391 without downloads: a data YAML (or its parsed dict) -> dict with 'names' (dict),
    'nc', and absolute 'train'/'val'/'test' paths.  A relative 'path' is taken relative to the YAML's folder
    (the reference resolves it under its settings' datasets_dir, which this package does not have)."""
    import yaml

    if isinstance(dataset, dict):
        data, root = dict(dataset), Path.cwd()
    else:
        file = Path(dataset)
        if file.is_dir():
            file = find_dataset_yaml(file)
        if not file.is_file():
            raise FileNotFoundError(f"dataset '{dataset}' not found")
        with open(file, errors="ignore", encoding="utf-8") as f:
            data = yaml.safe_load(f) or {}
        data["yaml_file"] = str(file)
        root = file.parent
    for k in ("train", "val"):
        if k not in data:
            if k != "val" or "validation" not in data:
                raise SyntaxError(f"{dataset} '{k}:' key missing: 'train' and 'val' are required in all data YAMLs")
            data["val"] = data.pop("validation")
    if "names" not in data and "nc" not in data:
        raise SyntaxError(f"{dataset}: either 'names' or 'nc' is required in data YAMLs")
    if "names" in data and "nc" in data and len(data["names"]) != data["nc"]:
        raise SyntaxError(f"{dataset}: 'names' length {len(data['names'])} and 'nc: {data['nc']}' must match")
    if "names" not in data:
        data["names"] = [f"class_{i}" for i in range(data["nc"])]
    else:
        data["nc"] = len(data["names"])
    names = data["names"]
    data["names"] = dict(enumerate(names)) if isinstance(names, (list, tuple)) else {int(k): v for k, v in names.items()}
    path = Path(data.get("path") or root)
    if not path.is_absolute():
        path = (root / path).resolve()
    data["path"] = path
    for k in ("train", "val", "test", "minival"):
        if data.get(k):
            if isinstance(data[k], str):
                x = (path / data[k]).resolve()
                if not x.exists() and data[k].startswith("../"):
                    x = (path / data[k][3:]).resolve()
                data[k] = str(x)
            else:
                data[k] = [str((path / x).resolve()) for x in data[k]]
    val = data.get("val")
    for v in val if isinstance(val, list) else [val]:
        if v and not Path(v).exists():
            raise FileNotFoundError(f"dataset '{dataset}' val images not found, missing path '{v}'")
    return data


# ----------------------------------------------------------------------------------------- files and labels
def get_img_files(img_path) -> list[str]:
    """BaseDataset.get_img_files (U/data/base.py:106-130): a directory (recursive), a *.txt list of images
    ('./' relative to the list's folder), or a list of those; sorted, image suffixes only."""
    f = []
    for p in img_path if isinstance(img_path, list) else [img_path]:
        p = Path(p)
        if p.is_dir():
            f += glob.glob(str(p / "**" / "*.*"), recursive=True)
        elif p.is_file():
            parent = str(p.parent) + os.sep
            f += [x.replace("./", parent) if x.startswith("./") else x for x in p.read_text().strip().splitlines()]
        else:
            raise FileNotFoundError(f"{p} does not exist")
    im_files = sorted(x.replace("/", os.sep) for x in f if x.split(".")[-1].lower() in IMG_FORMATS)
    if not im_files:
        raise FileNotFoundError(f"no images found in {img_path}")
    return im_files


def img2label_paths(img_paths) -> list[str]:
    """U/data/utils.py:44-47: /images/ -> /labels/, suffix -> .txt."""
    sa, sb = f"{os.sep}images{os.sep}", f"{os.sep}labels{os.sep}"
    return [sb.join(x.rsplit(sa, 1)).rsplit(".", 1)[0] + ".txt" for x in img_paths]


def _exif_hw(im) -> tuple[int, int]:
    """exif_size (U/data/utils.py:58-69) as (h, w)."""
    w, h = im.size
    if im.format == "JPEG":
        try:
            rot = im.getexif().get(274, None)
            if rot in {6, 8}:
                w, h = h, w
        except Exception:  # noqa: BLE001 - a broken EXIF block leaves the size as stored, like the reference
            pass
    return h, w


def _segments2boxes(segments) -> np.ndarray:
    """U/utils/ops.py:603-617: polygon -> xywh of its extent."""
    b = np.array([[s[:, 0].min(), s[:, 1].min(), s[:, 0].max(), s[:, 1].max()] for s in segments])
    y = np.empty_like(b)
    y[:, 0] = (b[:, 0] + b[:, 2]) / 2
    y[:, 1] = (b[:, 1] + b[:, 3]) / 2
    y[:, 2] = b[:, 2] - b[:, 0]
    y[:, 3] = b[:, 3] - b[:, 1]
    return y


def verify_image_label(im_file: str, lb_file: str, num_cls: int):
    """U/data/utils.py:97-165 for detect labels -> (hw, lb float32 [n, 5] cls+xywhn, msg) or (None, None, msg)
    for a corrupt pair.  A missing or empty label file is a background image (0 labels)."""
    from PIL import Image

    try:
        with Image.open(im_file) as im:
            im.verify()
            shape = _exif_hw(im)
            fmt = (im.format or "").lower()
        if not (shape[0] > 9 and shape[1] > 9):
            raise ValueError(f"image size {shape} <10 pixels")
        if fmt not in IMG_FORMATS:
            raise ValueError(f"invalid image format {fmt}")
        msg = ""
        lb = np.zeros((0, 5), dtype=np.float32)
        if os.path.isfile(lb_file):
            with open(lb_file) as f:
                rows = [x.split() for x in f.read().strip().splitlines() if len(x)]
            if any(len(x) > 6 for x in rows):  # segments
                classes = np.array([x[0] for x in rows], dtype=np.float32)
                segs = [np.array(x[1:], dtype=np.float32).reshape(-1, 2) for x in rows]
                rows = np.concatenate((classes.reshape(-1, 1), _segments2boxes(segs)), 1)
            lb = np.array(rows, dtype=np.float32).reshape(-1, 5) if len(rows) else lb
            if nl := len(lb):
                if lb.shape[1] != 5:
                    raise ValueError(f"labels require 5 columns, {lb.shape[1]} columns detected")
                if lb[:, 1:].max() > 1:
                    raise ValueError("non-normalized or out of bounds coordinates")
                if lb.min() < 0:
                    raise ValueError("negative label values")
                if lb[:, 0].max() > num_cls:  # the reference's bound (max_cls <= num_cls)
                    raise ValueError(f"label class {int(lb[:, 0].max())} exceeds dataset class count {num_cls}")
                _, i = np.unique(lb, axis=0, return_index=True)
                if len(i) < nl:  # duplicate rows removed (in np.unique's sorted order, like the reference)
                    lb = lb[i]
                    msg = f"{im_file}: {nl - len(i)} duplicate labels removed"
        return shape, lb, msg
    except Exception as e:  # noqa: BLE001 - a corrupt pair is skipped with a message (verify_image_label)
        return None, None, f"{im_file}: ignoring corrupt image/label: {e}"


def load_bgr(im_file: str) -> np.ndarray:
    """cv2.imread(f) (IMREAD_COLOR: 3-channel BGR uint8, EXIF orientation applied) through PIL; an existing
    <image>.npy next to the file is used instead, as BaseDataset.load_image does (U/data/base.py:153-163)."""
    npy = Path(im_file).with_suffix(".npy")
    if npy.exists():
        im = np.load(npy, allow_pickle=False)
        if im.dtype == np.uint8 and im.ndim == 3 and im.shape[2] == 3:
            return im
    from PIL import Image, ImageOps

    with Image.open(im_file) as im:
        if im.format == "JPEG":
            im = ImageOps.exif_transpose(im)
        rgb = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(rgb[..., ::-1])


# ------------------------------------------------------------------------------------------------ dataset
class YOLOValDataset:
    """The val-mode YOLODataset (augment=False, pad=0.5, rect per Model.val's default, U/engine/model.py:636-637).

    ``labels[i]`` = {"im_file", "shape" (h, w), "cls" [n, 1], "bboxes" [n, 4] normalized xywh}, in the
    rect order; iterating yields host batches (see ``batches``)."""

    def __init__(self, img_path, imgsz=640, batch_size=16, stride=32, rect=True, pad=0.5, single_cls=False,
                 classes=None, num_cls=80, workers=8):
        self.imgsz, self.batch_size, self.stride = int(imgsz), int(batch_size), int(stride)
        self.rect, self.pad, self.workers = bool(rect), float(pad), max(1, int(workers))
        im_files = get_img_files(img_path)
        lb_files = img2label_paths(im_files)
        self.msgs = []
        labels = []
        with ThreadPoolExecutor(self.workers) as ex:
            res = list(ex.map(lambda a: verify_image_label(*a, num_cls), zip(im_files, lb_files)))
        for f, (shape, lb, msg) in zip(im_files, res):
            if msg:
                self.msgs.append(msg)
            if shape is not None:
                labels.append({"im_file": f, "shape": shape, "cls": lb[:, 0:1], "bboxes": lb[:, 1:]})
        if not labels:
            raise FileNotFoundError(f"no valid images in {img_path}")
        if classes is not None:  # update_labels (U/data/base.py:132-149)
            keep = np.array(classes).reshape(1, -1)
            for lb in labels:
                j = (lb["cls"] == keep).any(1)
                lb["cls"], lb["bboxes"] = lb["cls"][j], lb["bboxes"][j]
        if single_cls:
            for lb in labels:
                lb["cls"][:, 0] = 0
        self.labels = labels
        self.batch_shapes = None
        if self.rect:
            self._set_rectangle()

    @property
    def im_files(self):
        return [lb["im_file"] for lb in self.labels]

    def __len__(self):
        return len(self.labels)

    def _set_rectangle(self):
        """U/data/base.py:261-284."""
        n = len(self.labels)
        bi = np.floor(np.arange(n) / self.batch_size).astype(int)
        nb = bi[-1] + 1
        s = np.array([lb["shape"] for lb in self.labels])
        ar = s[:, 0] / s[:, 1]
        irect = ar.argsort()
        self.labels = [self.labels[i] for i in irect]
        ar = ar[irect]
        shapes = [[1, 1]] * nb
        for i in range(nb):
            ari = ar[bi == i]
            mini, maxi = ari.min(), ari.max()
            if maxi < 1:
                shapes[i] = [maxi, 1]
            elif mini > 1:
                shapes[i] = [1, 1 / mini]
        self.batch_shapes = np.ceil(np.array(shapes) * self.imgsz / self.stride + self.pad).astype(int) * self.stride
        self.batch = bi

    def geometry(self, ori_hw, index):
        """load_image's long-side resize + LetterBox(scaleup=False) -> (resized hw, letterbox (H, W), top, left)."""
        h0, w0 = ori_hw
        r = self.imgsz / max(h0, w0)
        h, w = (min(math.ceil(h0 * r), self.imgsz), min(math.ceil(w0 * r), self.imgsz)) if r != 1 else (h0, w0)
        if self.rect:
            new_shape = tuple(int(v) for v in self.batch_shapes[self.batch[index]])
        else:
            new_shape = (self.imgsz, self.imgsz)
        rr = min(min(new_shape[0] / h, new_shape[1] / w), 1.0)
        new_unpad = int(round(w * rr)), int(round(h * rr))
        if new_unpad != (w, h):
            raise NotImplementedError("LetterBox would resize a second time; the fused val letterbox covers "
                                      "rect/square val shapes only")
        dw, dh = (new_shape[1] - w) / 2, (new_shape[0] - h) / 2
        top, left = int(round(dh - 0.1)), int(round(dw - 0.1))
        return (h, w), new_shape, top, left

    def _item(self, index, im):
        """One image's host-side val sample (get_image_and_label + LetterBox + Format)."""
        lb = self.labels[index]
        ori = im.shape[:2]
        (h, w), (H, W), top, left = self.geometry(ori, index)
        box = lb["bboxes"].astype(np.float32).copy()  # Instances: xywh normalized, float32
        if len(box):
            xyxy = np.empty_like(box)  # convert_bbox('xyxy')
            half = box[:, 2:] / 2
            xyxy[:, :2] = box[:, :2] - half
            xyxy[:, 2:] = box[:, :2] + half
            for k, sc in enumerate((w, h, w, h)):  # denormalize to the resized image, scale(1, 1), add_padding
                xyxy[:, k] *= sc
                xyxy[:, k] *= 1.0
                xyxy[:, k] += (left, top)[k % 2]
            box = np.empty_like(xyxy)  # Format: convert_bbox('xywh'), normalize by the letterboxed size
            box[:, 0] = (xyxy[:, 0] + xyxy[:, 2]) / 2
            box[:, 1] = (xyxy[:, 1] + xyxy[:, 3]) / 2
            box[:, 2] = xyxy[:, 2] - xyxy[:, 0]
            box[:, 3] = xyxy[:, 3] - xyxy[:, 1]
            box[:, [0, 2]] /= np.float32(W)
            box[:, [1, 3]] /= np.float32(H)
        return {"im_file": lb["im_file"], "img": im, "ori_shape": ori, "resized_shape": (h, w), "shape": (H, W),
                "top_left": (top, left), "ratio_pad": ((h / ori[0], w / ori[1]), (left, top)),
                "cls": lb["cls"].astype(np.float32), "bboxes": box}

    def batches(self):
        """Yields collated host batches: {"frames": [HWC uint8 BGR], "meta" int32 [b, 6] (h0, w0, h, w, top,
        left) for ydbl_letterbox, "shape" (H, W), "ori_shape", "ratio_pad", "im_file", "cls" [N], "bboxes" [N, 4]
        normalized xywh of the letterboxed image, "batch_idx" [N]}.  Images are decoded by a thread pool one batch
        ahead of the consumer."""
        n = len(self.labels)
        starts = list(range(0, n, self.batch_size))
        with ThreadPoolExecutor(self.workers) as ex, ThreadPoolExecutor(1) as ahead:
            def decode(s):
                return list(ex.map(load_bgr, [lb["im_file"] for lb in self.labels[s: s + self.batch_size]]))

            nxt = ahead.submit(decode, starts[0]) if starts else None
            for k, s in enumerate(starts):
                ims = nxt.result()
                nxt = ahead.submit(decode, starts[k + 1]) if k + 1 < len(starts) else None
                items = [self._item(s + j, im) for j, im in enumerate(ims)]
                shapes = {it["shape"] for it in items}
                if len(shapes) != 1:
                    raise RuntimeError(f"images of one batch letterbox to different shapes {sorted(shapes)}")
                yield {
                    "frames": [it["img"] for it in items],
                    "meta": np.array([[*it["ori_shape"], *it["resized_shape"], *it["top_left"]] for it in items],
                                     dtype=np.int32),
                    "shape": shapes.pop(),
                    "ori_shape": [it["ori_shape"] for it in items],
                    "ratio_pad": [it["ratio_pad"] for it in items],
                    "im_file": [it["im_file"] for it in items],
                    "cls": np.concatenate([it["cls"].reshape(-1) for it in items]),
                    "bboxes": np.concatenate([it["bboxes"].reshape(-1, 4) for it in items]),
                    "batch_idx": np.concatenate([np.full(len(it["cls"]), j, dtype=np.float32)
                                                 for j, it in enumerate(items)]),
                }
