"""Host side of the dataset-backed val (ydbl.engine.dataset) against the oracle's restatement of the reference's
val data pipeline (oracle/dataset.py): files, labels, rect batch shapes, letterbox geometry, label transforms and
the native-space labels.  The GPU letterbox and the full .val() loop are in test_gpu_val.py."""

import numpy as np
import pytest
import torch

from dataset_util import make_dataset


@pytest.fixture(scope="module")
def ds_yaml(tmp_path_factory):
    return make_dataset(tmp_path_factory.mktemp("ds"))


def test_check_det_dataset(ds_yaml, tmp_path):
    from ydbl.engine.dataset import check_det_dataset

    d = check_det_dataset(ds_yaml)
    assert d["nc"] == 3 and d["names"] == {0: "c0", 1: "c1", 2: "c2"}
    assert d["val"] == str((ds_yaml.parent / "images" / "val").resolve())
    assert check_det_dataset(ds_yaml.parent)["val"] == d["val"]  # dataset folder -> its YAML
    bad = tmp_path / "bad.yaml"
    bad.write_text("val: x\nnames: [a]\n")
    with pytest.raises(SyntaxError):
        check_det_dataset(bad)  # 'train' is required
    bad.write_text("train: x\nval: x\nnc: 2\nnames: [a]\n")
    with pytest.raises(SyntaxError):
        check_det_dataset(bad)  # names / nc mismatch
    bad.write_text("train: x\nval: missing_dir\nnc: 2\n")
    with pytest.raises(FileNotFoundError):
        check_det_dataset(bad)


def test_img2label_paths():
    from ydbl.engine.dataset import img2label_paths

    assert img2label_paths(["/d/images/val/a.b.png", "/images/x/images/y.jpg"]) == \
        ["/d/labels/val/a.b.txt", "/images/x/labels/y.txt"]


@pytest.mark.parametrize("batch,imgsz,rect", [(4, 640, True), (3, 320, True), (16, 640, True), (4, 416, False)])
def test_dataset_matches_oracle(ds_yaml, batch, imgsz, rect):
    from oracle.dataset import ValData, data_yaml
    from oracle.letterbox import resize_linear_u8
    from ydbl.engine.dataset import YOLOValDataset, check_det_dataset
    from ydbl.engine.validator import native_labels

    d = check_det_dataset(ds_yaml)
    ds = YOLOValDataset(d["val"], imgsz=imgsz, batch_size=batch, rect=rect, num_cls=d["nc"], workers=2)
    ref = ValData(data_yaml(ds_yaml)["val"], imgsz, batch, num_cls=3, rect=rect)
    assert ds.im_files == [it["im_file"] for it in ref.items]
    assert len(ds) == 10  # corrupt.jpg and the out-of-range class are skipped, notes.txt is not an image
    assert any("ignoring corrupt" in m for m in ds.msgs) and any("duplicate" in m for m in ds.msgs)
    hbs = list(ds.batches())
    assert len(hbs) == len(ref)
    for k, hb in enumerate(hbs):
        rb = ref.batch(k)
        assert hb["shape"] == tuple(rb["img"].shape[2:])
        assert hb["ori_shape"] == rb["ori_shape"] and hb["ratio_pad"] == rb["ratio_pad"]
        assert torch.equal(torch.from_numpy(hb["cls"]), rb["cls"].reshape(-1))
        assert torch.equal(torch.from_numpy(hb["batch_idx"]), rb["batch_idx"])
        assert torch.equal(torch.from_numpy(hb["bboxes"]).reshape(-1, 4), rb["bboxes"].reshape(-1, 4))
        # the one-pass letterbox (resize to meta's size, place at (top, left)) == load_image + LetterBox
        H, W = hb["shape"]
        for j, (f, m) in enumerate(zip(hb["frames"], hb["meta"])):
            canvas = np.full((H, W, 3), 114, np.uint8)
            r = f if (m[2], m[3]) == f.shape[:2] else resize_linear_u8(f, int(m[2]), int(m[3]))
            canvas[m[4]: m[4] + m[2], m[5]: m[5] + m[3]] = r
            assert np.array_equal(canvas[..., ::-1].transpose(2, 0, 1), rb["img"][j].numpy())
        # native-space labels (val.py:104-115)
        from oracle.dataset import scale_boxes_ratio_pad
        from oracle.ops import xywh2xyxy

        nat = native_labels(hb)
        for si in range(len(hb["frames"])):
            idx = rb["batch_idx"] == si
            if idx.any():
                bb = xywh2xyxy(rb["bboxes"][idx]) * torch.tensor((H, W))[[1, 0, 1, 0]]
                scale_boxes_ratio_pad(bb, rb["ori_shape"][si], rb["ratio_pad"][si])
                assert torch.equal(nat[torch.from_numpy(hb["batch_idx"]) == si], bb)


def test_rect_shapes_known_values(ds_yaml):
    """set_rectangle arithmetic: ceil(shape * imgsz / stride + 0.5) * stride per batch."""
    from ydbl.engine.dataset import YOLOValDataset

    ds = YOLOValDataset(ds_yaml.parent / "images" / "val", imgsz=640, batch_size=16, num_cls=3, workers=1)
    ar = sorted(h / w for h, w in [lb["shape"] for lb in ds.labels])
    assert (ds.batch_shapes == np.ceil(np.array([[1, 1]]) * 20 + 0.5).astype(int) * 32).all()  # mixed ratios
    assert ar[0] < 1 < ar[-1]
    ds2 = YOLOValDataset(ds_yaml.parent / "images" / "val", imgsz=640, batch_size=2, num_cls=3, workers=1)
    first = ds2.labels[0]["shape"], ds2.labels[1]["shape"]
    maxi = max(s[0] / s[1] for s in first)
    assert tuple(ds2.batch_shapes[0]) == (int(np.ceil(maxi * 20 + 0.5)) * 32, 672)


def test_single_cls_and_classes(ds_yaml):
    from ydbl.engine.dataset import YOLOValDataset

    img = ds_yaml.parent / "images" / "val"
    a = YOLOValDataset(img, imgsz=320, batch_size=4, num_cls=3, single_cls=True, workers=1)
    assert all((lb["cls"] == 0).all() for lb in a.labels)
    b = YOLOValDataset(img, imgsz=320, batch_size=4, num_cls=3, classes=[1], workers=1)
    assert all((lb["cls"] == 1).all() for lb in b.labels)
