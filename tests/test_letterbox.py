"""LetterBox geometry and the oracle's cv2 INTER_LINEAR restatement (CPU); the GPU kernel vs the oracle
(bit-exact) and the ndarray predict path (gpu)."""

from pathlib import Path

import numpy as np
import pytest
import torch

SHAPES = [(480, 640), (720, 1280), (333, 517), (1280, 1280), (200, 300), (640, 640), (1080, 1920), (17, 999),
          (641, 639)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("auto", [False, True])
def test_geometry_product_matches_oracle(shape, auto):
    from oracle.letterbox import letterbox_geometry as ref
    from ydbl.engine.preprocess import letterbox_geometry

    for imgsz in [(640, 640), (1280, 1280), (320, 480)]:
        assert letterbox_geometry(shape, imgsz, auto=auto) == ref(shape, imgsz, auto=auto)


def test_geometry_known_values():
    from ydbl.engine.preprocess import letterbox_geometry

    # r = 1: nothing resized, 160 rows of padding split 80/80 (auto=False) or 0 (auto: 160 % 32 == 0)
    assert letterbox_geometry((480, 640), 640) == (480, 640, 80, 80, 0, 0)
    assert letterbox_geometry((480, 640), 640, auto=True) == (480, 640, 0, 0, 0, 0)
    # 1080p: r = 1/3, unpad 360x640, dh = 280 -> auto: 280 % 32 = 24 -> 12 / 12
    assert letterbox_geometry((1080, 1920), 640, auto=True) == (360, 640, 12, 12, 0, 0)
    # odd padding: round(dh -/+ 0.1) puts the extra row at the bottom
    assert letterbox_geometry((331, 640), 640)[2:4] == (154, 155)


def test_resize_identity_constant_and_area_shortcut():
    from oracle.letterbox import resize_linear_u8

    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    const = np.full((37, 53, 3), 77, dtype=np.uint8)
    for dh, dw in [(74, 106), (20, 30), (37, 26), (100, 17)]:
        assert (resize_linear_u8(const, dh, dw) == 77).all()
    big = rng.integers(0, 256, (64, 48, 3), dtype=np.uint8)
    half = resize_linear_u8(big, 32, 24)
    s = big.astype(int)
    assert (half == ((s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2)).all()
    # bilinear stays within the local min/max of its 2x2 source neighbourhood
    up = resize_linear_u8(img, 90, 120)
    assert up.min() >= img.min() and up.max() <= img.max()


def test_preprocess_layout():
    from oracle.letterbox import preprocess

    img = np.zeros((64, 96, 3), dtype=np.uint8)
    img[..., 0] = 10  # B
    img[..., 2] = 250  # R
    x = preprocess([img], imgsz=(96, 96), stride=32, pt=False)
    assert x.shape == (1, 3, 96, 96) and x.dtype == np.float32
    assert x[0, 0, 48, 48] == np.float32(250) / np.float32(255)  # R first
    assert x[0, 2, 48, 48] == np.float32(10) / np.float32(255)
    assert x[0, 1, 0, 0] == np.float32(114) / np.float32(255)  # border row


def _frames(shapes, seed):
    rng = np.random.default_rng(seed)
    out = []
    for h, w in shapes:
        # smooth content + noise so interpolation weights matter
        yy, xx = np.mgrid[0:h, 0:w]
        base = (np.stack([xx * 3 + yy, xx + yy * 2, xx * yy // 7], -1) % 256).astype(np.int64)
        out.append(np.clip(base + rng.integers(-20, 21, (h, w, 3)), 0, 255).astype(np.uint8))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("shapes,imgsz", [
    ([(480, 640)] * 3, (640, 640)),
    ([(1080, 1920)] * 2, (640, 640)),
    ([(1280, 1280), (333, 517), (200, 300), (640, 640)], (640, 640)),
    ([(17, 999), (641, 639)], (320, 480)),
    ([(2560, 1440)], (1280, 1280)),
])
def test_letterbox_kernel_bit_exact(shapes, imgsz):
    from oracle.letterbox import preprocess
    from ydbl.engine.preprocess import letterbox_batch

    frames = _frames(shapes, seed=len(shapes))
    ref = torch.from_numpy(preprocess(frames, imgsz, stride=32, pt=True))
    got = letterbox_batch(frames, imgsz, stride=32, device="cuda").cpu()
    assert got.shape == ref.shape
    assert torch.equal(got, ref), (got - ref).abs().max()


@pytest.mark.gpu
def test_predict_frames_matches_tensor_path():
    """ndarray frames through the GPU letterbox give the tensor path's detections on the oracle-letterboxed
    batch, mapped back with scale_boxes (U/utils/ops.py:92-127)."""
    from oracle.letterbox import preprocess
    from ydbl import YOLO
    from ydbl.engine.preprocess import scale_boxes
    from ydbl.utils.synthetic import blob_images

    m = YOLO("yolov13n_DBL.yaml", nc=3)
    x = blob_images(2, 256, seed=11)  # [2,3,256,256] 0..1 RGB
    frames = [np.ascontiguousarray((x[i].permute(1, 2, 0).numpy()[:, :, ::-1] * 255).round().astype(np.uint8))
              for i in range(2)]
    frames = [np.ascontiguousarray(np.concatenate([f, f[:, :64]], 1)) for f in frames]  # 256x320
    res = m.predict(frames, imgsz=320, conf=0.05)
    xb = torch.from_numpy(preprocess(frames, (320, 320), stride=32, pt=True))
    s = m.session(2, xb.shape[2], xb.shape[3], conf=0.05, clip=False)
    det, cnt = s(xb.cuda())
    for i in range(2):
        ref = det[i, : int(cnt[i])].clone()
        scale_boxes(xb.shape[2:], ref, frames[i].shape[:2])
        assert torch.equal(res[i].boxes.data, ref)
        assert res[i].orig_shape == frames[i].shape[:2]


def _write_pngs(tmp_path, frames, names):
    from PIL import Image

    paths = []
    for f, n in zip(frames, names):
        p = tmp_path / n
        Image.fromarray(np.ascontiguousarray(f[:, :, ::-1])).save(p)  # BGR frame -> RGB file
        paths.append(p)
    return paths


def test_sources_file_collection(tmp_path):
    """LoadImagesAndVideos file rules (U/data/loaders.py:328-351): dir = sorted *.*, glob, *.txt relative to its
    folder, images only; PIL / ndarray sources decode to the BGR frames cv2 would give (lossless PNG)."""
    from PIL import Image

    from ydbl.engine.sources import frames_from_images, image_files

    frames = _frames([(40, 60), (30, 20), (50, 50)], seed=5)
    paths = _write_pngs(tmp_path, frames, ["b.png", "a.png", "c.png"])
    (tmp_path / "notes.json").write_text("{}")
    want = [str(tmp_path / n) for n in ("a.png", "b.png", "c.png")]
    assert image_files(tmp_path) == want
    assert image_files(str(tmp_path / "*.png")) == want
    (tmp_path / "list.txt").write_text("c.png\nb.png\n")
    assert image_files(tmp_path / "list.txt") == [want[1], want[2]]  # list entries sorted, as the reference
    with pytest.raises(FileNotFoundError):
        image_files(tmp_path / "missing.png")
    ps, got = frames_from_images([Image.open(paths[0]), str(paths[1]), frames[2]])
    assert ps == [str(paths[0]), str(paths[1]), "image2.jpg"]
    for g, f in zip(got, frames):
        assert g.dtype == np.uint8 and np.array_equal(g, f)


@pytest.mark.gpu
def test_predict_file_dir_glob_pil_sources(tmp_path):
    """predict() on a file, a directory, a glob, a *.txt list and PIL images gives the ndarray-frame path's
    detections (same frames, same batch composition), with the file paths on the Results."""
    from PIL import Image

    from ydbl import YOLO
    from ydbl.utils.synthetic import blob_images, load_trained

    m = YOLO("yolov13n_DBL.yaml", nc=3)
    load_trained(m.model, Path(__file__).resolve().parent / "golden" / "trained_yolov13n_DBL_nc3.npz")
    x = blob_images(2, 256, seed=11)
    frames = [np.ascontiguousarray((x[i].permute(1, 2, 0).numpy()[:, :, ::-1] * 255).round().astype(np.uint8))
              for i in range(2)]
    paths = _write_pngs(tmp_path, frames, ["f0.png", "f1.png"])
    one = [m.predict(f, imgsz=256, conf=0.05)[0] for f in frames]  # batch of one frame each
    both = m.predict(frames, imgsz=256, conf=0.05)
    assert sum(len(r.boxes.data) for r in both) > 0
    cases = [(m.predict(str(paths[0]), imgsz=256, conf=0.05), one[:1]),
             (m.predict(tmp_path, imgsz=256, conf=0.05), one),
             (list(m.predict(str(tmp_path / "*.png"), imgsz=256, conf=0.05, stream=True)), one),
             (m.predict(tmp_path, imgsz=256, conf=0.05, batch=2), both),
             (m.predict([Image.open(p) for p in paths], imgsz=256, conf=0.05), both),
             (m.predict([str(p) for p in paths], imgsz=256, conf=0.05), both)]
    (tmp_path / "l.txt").write_text("f1.png\n")
    cases.append((m.predict(tmp_path / "l.txt", imgsz=256, conf=0.05), one[1:]))
    for got, want in cases:
        assert len(got) == len(want)
        for g, w in zip(got, want):
            assert torch.equal(g.boxes.data, w.boxes.data)
    assert m.predict(tmp_path, imgsz=256, conf=0.05)[1].path == str(paths[1])


@pytest.mark.gpu
def test_session_cache_is_bounded():
    """Model._sessions is an LRU of MAX_SESSIONS entries: predict() over many batch sizes does not keep every
    compiled session (and its HBM) alive."""
    from ydbl import YOLO

    m = YOLO("yolov13n_DBL.yaml", nc=3)
    for b in range(1, m.MAX_SESSIONS + 3):
        m.predict(torch.rand(b, 3, 64, 64), conf=0.5)
    assert len(m._sessions) == m.MAX_SESSIONS
    keys = list(m._sessions)
    assert [k[0] for k in keys] == list(range(3, m.MAX_SESSIONS + 3))
    m.predict(torch.rand(3, 3, 64, 64), conf=0.5)  # hit: becomes most recent
    assert list(m._sessions)[-1][0] == 3
