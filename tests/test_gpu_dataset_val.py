"""Dataset-backed .val(data=<yaml>) on the GPU against the oracle's CPU restatement of the reference's val loop
(oracle/dataset.py): YOLO-format files with rect batches, letterboxed by ydbl_letterbox, matched in native image
space after scale_boxes(ratio_pad) (U/models/yolo/detect/val.py:104-123, :230-248)."""

import shutil

import numpy as np
import pytest
import torch

from dataset_util import make_dataset

pytestmark = pytest.mark.gpu


def _pseudo_gt_dataset(root, o, imgsz, conf=0.1):
    """Images from dataset_util, labels = the oracle's own detections (conf `conf`) in native space."""
    from oracle.dataset import ValData, data_yaml, scale_boxes_ratio_pad
    from oracle.ops import non_max_suppression

    y = make_dataset(root, labels={}, edge_cases=False)
    vd = ValData(data_yaml(y)["val"], imgsz, 4, num_cls=3)
    for k in range(len(vd)):
        bt = vd.batch(k)
        with torch.no_grad():
            yy, _ = o(bt["img"].float() / 255)
        for si, p in enumerate(non_max_suppression(yy, conf, 0.7)):
            p = p.clone()
            scale_boxes_ratio_pad(p[:, :4], bt["ori_shape"][si], bt["ratio_pad"][si])
            h0, w0 = bt["ori_shape"][si]
            xc, yc = (p[:, 0] + p[:, 2]) / 2 / w0, (p[:, 1] + p[:, 3]) / 2 / h0
            bw, bh = (p[:, 2] - p[:, 0]) / w0, (p[:, 3] - p[:, 1]) / h0
            rows = [f"{int(c)} {a:.6f} {b:.6f} {cc:.6f} {d:.6f}" for c, a, b, cc, d in
                    zip(p[:, 5].tolist(), xc.tolist(), yc.tolist(), bw.tolist(), bh.tolist()) if cc > 0 and d > 0]
            lf = bt["im_file"][si].replace("/images/", "/labels/").rsplit(".", 1)[0] + ".txt"
            open(lf, "w").write("\n".join(rows))
    return y


def _metrics(stats):
    from ydbl.utils.metrics import DetMetrics

    m = DetMetrics()
    m.process(stats["tp"], stats["conf"], stats["pred_cls"], stats["target_cls"])
    return m.box.map50, m.box.map


@pytest.mark.parametrize("half", [False, True])
def test_val_yaml_matches_oracle(tmp_path, golden_dir, half):
    from oracle.dataset import ValData, data_yaml, validate
    from parity_util import build_pair
    from ydbl.engine.dataset import YOLOValDataset, check_det_dataset
    from ydbl.engine.preprocess import letterbox_frames

    imgsz, batch = 320, 4
    p, o = build_pair("n", 3, golden_dir)
    y = _pseudo_gt_dataset(tmp_path / "ds", o, imgsz)
    # letterboxed batches: the one-pass GPU letterbox == load_image + LetterBox, bit for bit
    d = check_det_dataset(y)
    ds = YOLOValDataset(d["val"], imgsz=imgsz, batch_size=batch, num_cls=3, workers=2)
    ref = ValData(data_yaml(y)["val"], imgsz, batch, num_cls=3)
    stats_ref, ref_imgs = validate(o, ref)
    for hb, rimg in zip(ds.batches(), ref_imgs):
        got = letterbox_frames(hb["frames"], hb["meta"], *hb["shape"], device="cuda").cpu()
        assert torch.equal(got, rimg.float() / 255)
    m = p.val(data=str(y), imgsz=imgsz, batch=batch, half=half)
    m50_ref, m_ref = _metrics(stats_ref)
    n_gt = len(stats_ref["target_cls"])
    print(f"val(data=yaml) {'fp16' if half else 'fp32'}: mAP50 {m.box.map50:.4f} (oracle {m50_ref:.4f}), "
          f"mAP50-95 {m.box.map:.4f} (oracle {m_ref:.4f}), {n_gt} labels")
    assert n_gt > 100 and m50_ref > 0.8
    tol = 0.1 if half else 0.01
    assert abs(m.box.map50 - m50_ref) <= tol and abs(m.box.map - m_ref) <= tol


def test_val_image_folder_and_square(tmp_path, golden_dir):
    """data=<image folder> (names from the model) and rect=False (square imgsz LetterBox) run the same pipeline."""
    from oracle.dataset import ValData, validate
    from parity_util import build_pair

    p, o = build_pair("n", 3, golden_dir)
    y = _pseudo_gt_dataset(tmp_path / "ds", o, 256)
    img_dir = y.parent / "images" / "val"
    stats_ref, _ = validate(o, ValData(str(img_dir), 256, 3, num_cls=3, rect=False))
    m = p.val(data=str(img_dir), imgsz=256, batch=3, rect=False)
    m50_ref, _ = _metrics(stats_ref)
    assert abs(m.box.map50 - m50_ref) <= 0.01
    shutil.rmtree(tmp_path / "ds")
