"""Synthetic YOLO-format datasets on disk for the .val(data=...) tests (test infrastructure)."""

from __future__ import annotations

from pathlib import Path

import numpy as np

# (h, w): landscape / portrait / square, down- and up-scaled by load_image, odd sizes, the 2x area shortcut
SHAPES = [(480, 640), (640, 480), (360, 640), (500, 500), (1024, 768), (300, 200), (720, 1280), (200, 600),
          (1280, 1280), (333, 517)]


def blob_bgr(h, w, seed):
    """A uint8 BGR frame with a few bright blobs on a textured background."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = 40 + 20 * np.sin(xx / 17.0)[..., None] * np.cos(yy / 23.0)[..., None] * np.ones(3, np.float32)
    for _ in range(int(rng.integers(4, 10))):
        cy, cx = rng.uniform(0.1, 0.9) * h, rng.uniform(0.1, 0.9) * w
        ry, rx = rng.uniform(0.04, 0.2) * h, rng.uniform(0.04, 0.2) * w
        col = rng.uniform(60, 255, 3)
        m = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
        img[m] = col
    img += rng.normal(0, 4, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def write_png(path: Path, bgr: np.ndarray):
    from PIL import Image

    path.parent.mkdir(parents=True, exist_ok=True)
    Image.fromarray(np.ascontiguousarray(bgr[..., ::-1])).save(path)


def make_dataset(root: Path, shapes=SHAPES, nc=3, seed=0, labels=None, edge_cases=True) -> Path:
    """images/val/*.png + labels/val/*.txt + data.yaml under root; returns the YAML path.

    labels: optional {stem: [[cls, x, y, w, h], ...]} (normalized xywh); default random boxes.  With
    edge_cases: a duplicated label row, a segment-format label, an empty and a missing label file, a corrupt
    image and an out-of-range class (both skipped by verify_image_label)."""
    rng = np.random.default_rng(seed)
    img_dir, lb_dir = root / "images" / "val", root / "labels" / "val"
    img_dir.mkdir(parents=True, exist_ok=True)
    lb_dir.mkdir(parents=True, exist_ok=True)
    for i, (h, w) in enumerate(shapes):
        stem = f"im{i:03d}"
        write_png(img_dir / f"{stem}.png", blob_bgr(h, w, seed * 100 + i))
        if labels is not None:
            rows = labels.get(stem, [])
        else:
            n = int(rng.integers(1, 6))
            xy = rng.uniform(0.2, 0.8, (n, 2))
            wh = rng.uniform(0.05, 0.3, (n, 2))
            rows = np.concatenate([rng.integers(0, nc, (n, 1)), xy, wh], 1).tolist()
        text = "\n".join(f"{int(r[0])} " + " ".join(f"{v:.6f}" for v in r[1:]) for r in rows)
        if edge_cases and i == 1 and rows:
            text += "\n" + text.splitlines()[0]  # duplicate row
        if edge_cases and i == 2:
            text = "1 0.1 0.2 0.3 0.2 0.35 0.6 0.12 0.5\n" + text  # one polygon -> all rows as segments
            text = "\n".join(r if len(r.split()) > 5 else
                             "{} {a} {b} {c} {b} {c} {d} {a} {d}".format(
                                 r.split()[0], a=float(r.split()[1]) - float(r.split()[3]) / 2,
                                 b=float(r.split()[2]) - float(r.split()[4]) / 2,
                                 c=float(r.split()[1]) + float(r.split()[3]) / 2,
                                 d=float(r.split()[2]) + float(r.split()[4]) / 2)
                             for r in text.splitlines())
        if edge_cases and i == 3:
            text = ""  # empty label file: background image
        if not (edge_cases and i == 4):  # i == 4: missing label file
            (lb_dir / f"{stem}.txt").write_text(text)
    if edge_cases:
        (img_dir / "corrupt.jpg").write_bytes(b"\xff\xd8\xff\xe0 not really a jpeg")
        write_png(img_dir / "badcls.png", blob_bgr(100, 120, 7))
        (lb_dir / "badcls.txt").write_text(f"{nc + 5} 0.5 0.5 0.2 0.2\n")
        (img_dir / "notes.txt").write_text("not an image")
    names = "\n".join(f"  {k}: c{k}" for k in range(nc))
    y = root / "data.yaml"
    y.write_text(f"path: .\ntrain: images/val\nval: images/val\nnames:\n{names}\n")
    return y
