"""predict() sources other than tensors: image files, directories, globs, *.txt lists, PIL images, ndarrays.

Restates the reference's source dispatch for still images (U/data/build.py:159-215 check_source /
load_inference_source) and the two loaders that serve them:
- LoadImagesAndVideos (U/data/loaders.py:284-447) for a str / Path source: one file, a directory
  (its ``*.*`` entries, sorted), a glob pattern, or a ``*.txt`` file listing sources (relative to the
  txt's folder); image files only (IMG_FORMATS, U/data/utils.py:38), read like cv2.imread (BGR, EXIF
  orientation applied), yielded in batches of ``batch`` images;
- LoadPilAndNumpy (U/data/loaders.py:451-513) for PIL images / HWC BGR uint8 ndarrays and lists of
  them (a list of paths is opened as PIL images first, autocast_list U/data/loaders.py:641-655), one
  batch of everything.
Video files, streams, URLs and screenshots are outside the hot path and raise.
Decoding stays on the host (PIL); the letterbox, the network and NMS run on the GPU (engine/preprocess.py).
"""

from __future__ import annotations

import glob
import os
from pathlib import Path

import numpy as np

IMG_FORMATS = {"bmp", "dng", "jpeg", "jpg", "mpo", "png", "tif", "tiff", "webp", "pfm", "heic"}
VID_FORMATS = {"asf", "avi", "gif", "m4v", "mkv", "mov", "mp4", "mpeg", "mpg", "ts", "wmv", "webm"}


def _is_pil(x) -> bool:
    try:
        from PIL import Image
    except ImportError:  # pragma: no cover - Pillow is part of the image
        return False
    return isinstance(x, Image.Image)


def pil_to_bgr(im) -> np.ndarray:
    """LoadPilAndNumpy._single_check (U/data/loaders.py:493-502): RGB-convert, then channels reversed to BGR."""
    if im.mode != "RGB":
        im = im.convert("RGB")
    return np.ascontiguousarray(np.asarray(im)[:, :, ::-1])


def is_frame_source(source) -> bool:
    """PIL image, ndarray, or a list/tuple of those or of paths (check_source's from_img branch)."""
    if isinstance(source, np.ndarray) or _is_pil(source):
        return True
    return isinstance(source, (list, tuple)) and len(source) > 0 and all(
        isinstance(s, (np.ndarray, str, Path)) or _is_pil(s) for s in source)


def frames_from_images(source):
    """LoadPilAndNumpy (+ autocast_list for path elements): -> (paths, BGR uint8 HWC frames), one batch."""
    from PIL import Image

    items = list(source) if isinstance(source, (list, tuple)) else [source]
    paths, frames = [], []
    for i, im in enumerate(items):
        if isinstance(im, (str, Path)):
            s = str(im)
            if s.lower().startswith(("http://", "https://")):
                raise ValueError(f"URL sources need the network, which this framework does not use: {s}")
            with Image.open(s) as f:  # autocast_list opens paths as PIL images (no EXIF transpose there)
                paths.append(s)
                frames.append(pil_to_bgr(f))
            continue
        if _is_pil(im):
            paths.append(getattr(im, "filename", "") or f"image{i}.jpg")
            frames.append(pil_to_bgr(im))
        elif isinstance(im, np.ndarray):
            if im.ndim == 2:
                raise ValueError("ndarray sources must be HWC with 3 channels (BGR)")
            paths.append(f"image{i}.jpg")
            frames.append(np.ascontiguousarray(im))
        else:
            raise TypeError(f"type {type(im).__name__} is not a supported image type")
    return paths, frames


def image_files(path) -> list[str]:
    """LoadImagesAndVideos.__init__ file collection (U/data/loaders.py:328-351), images only."""
    parent = None
    if isinstance(path, (str, Path)) and Path(path).suffix == ".txt":
        parent = Path(path).parent
        path = Path(path).read_text().splitlines()
    files = []
    for p in sorted(map(str, path)) if isinstance(path, (list, tuple)) else [str(path)]:
        a = str(Path(p).absolute())
        if "*" in a:
            files.extend(sorted(glob.glob(a, recursive=True)))
        elif os.path.isdir(a):
            files.extend(sorted(glob.glob(os.path.join(a, "*.*"))))
        elif os.path.isfile(a):
            files.append(a)
        elif parent and (parent / p).is_file():
            files.append(str((parent / p).absolute()))
        else:
            raise FileNotFoundError(f"{p} does not exist")
    images = [f for f in files if f.split(".")[-1].lower() in IMG_FORMATS]
    videos = [f for f in files if f.split(".")[-1].lower() in VID_FORMATS]
    if videos:
        raise NotImplementedError(f"video sources are outside the inference hot path: {videos[:3]}")
    if not images:
        raise FileNotFoundError(f"No images found in {path}. Supported formats are:\nimages: {sorted(IMG_FORMATS)}")
    return images


def file_batches(source, batch: int = 1):
    """LoadImagesAndVideos.__next__ for images: yields (paths, BGR frames) batches of up to `batch` files."""
    from .dataset import load_bgr

    files = image_files(source)
    bs = max(int(batch), 1)
    for i in range(0, len(files), bs):
        chunk = files[i: i + bs]
        yield chunk, [load_bgr(f) for f in chunk]


def check_path_source(source) -> bool:
    """str / Path sources (check_source's first branch); streams, webcams, URLs and screenshots raise."""
    if not isinstance(source, (str, Path)):
        return False
    s = str(source)
    if s.isnumeric() or s.endswith(".streams") or s.lower() == "screen" or s.lower().startswith(
            ("https://", "http://", "rtsp://", "rtmp://", "tcp://")):
        raise NotImplementedError(f"stream / webcam / URL / screenshot sources are not supported: {s}")
    return True
