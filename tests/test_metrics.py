"""mAP machinery (host numpy restatement of U/utils/metrics.py / U/engine/validator.py) on
hand-checkable cases."""

import numpy as np
import torch


def test_box_iou_known_values():
    from oracle.metrics import box_iou

    a = torch.tensor([[0.0, 0.0, 10.0, 10.0]])
    b = torch.tensor([[0.0, 0.0, 10.0, 10.0], [5.0, 0.0, 15.0, 10.0], [20.0, 20.0, 30.0, 30.0]])
    iou = box_iou(a, b)[0]
    assert abs(iou[0].item() - 1.0) < 1e-6
    assert abs(iou[1].item() - 50.0 / 150.0) < 1e-6
    assert iou[2].item() == 0.0


def test_compute_ap_perfect_and_half():
    from ydbl.utils.metrics import compute_ap

    # the reference's sentinels (recall 1 -> precision 0) make a perfect curve 0.995 on the 101-point grid
    ap, _, _ = compute_ap(np.array([0.5, 1.0]), np.array([1.0, 1.0]))
    assert abs(ap - 0.995) < 1e-9
    # precision 1 up to recall 0.5, then the interpolation runs linearly to (1, 0): 0.5 + 0.25
    ap, _, _ = compute_ap(np.array([0.5]), np.array([1.0]))
    assert abs(ap - 0.75) < 1e-9


def test_match_predictions_greedy_unique():
    from oracle.metrics import IOUV, box_iou, match_predictions

    gt = torch.tensor([[0.0, 0.0, 10.0, 10.0]])
    gcls = torch.tensor([1.0])
    pred = torch.tensor([[0.0, 0.0, 10.0, 10.0], [0.0, 0.0, 10.0, 9.0], [0.0, 0.0, 10.0, 10.0]])
    pcls = torch.tensor([1.0, 1.0, 0.0])
    tp = match_predictions(pcls, gcls, box_iou(gt, pred), IOUV)
    assert tp[0].all()  # exact box, matched at every threshold
    assert not tp[1].any()  # the label is already taken by the better match
    assert not tp[2].any()  # wrong class


def test_ap_per_class_two_classes():
    from ydbl.utils.metrics import ap_per_class

    tp = np.array([[True] * 10, [False] * 10, [True] * 10])
    conf = np.array([0.9, 0.8, 0.7])
    pred_cls = np.array([0, 0, 1])
    target_cls = np.array([0, 1])
    *_, ap, classes = ap_per_class(tp, conf, pred_cls, target_cls)
    assert list(classes) == [0, 1]
    assert abs(ap[0, 0] - 0.995) < 1e-6 and abs(ap[1, 0] - 0.995) < 1e-6


def test_match_predictions_exact_tie_takes_larger_label():
    """The rule ydbl_match_predictions restates for exact IoU ties (numpy's reversed stable argsort on
    small match arrays): the detection matches the larger label index.  det0 overlaps both labels with
    IoU exactly 0.6 and takes label 1, which leaves label 0 to det1."""
    from oracle.metrics import IOUV, box_iou, match_predictions

    gt = torch.tensor([[0.0, 0.0, 10.0, 10.0], [5.0, 0.0, 15.0, 10.0]])
    gcls = torch.tensor([1.0, 1.0])
    pred = torch.tensor([[2.5, 0.0, 12.5, 10.0], [0.0, 0.0, 10.0, 10.0]])
    pcls = torch.tensor([1.0, 1.0])
    iou = box_iou(gt, pred)
    assert iou[0, 0] == iou[1, 0]
    tp = match_predictions(pcls, gcls, iou, IOUV)
    assert tp[0, :3].all() and not tp[0, 3:].any()
    assert tp[1].all()


def test_results_host_api(tmp_path):
    """Results/Boxes host API (U/engine/results.py): indexing, update+clip, save_txt, json/df, plot."""
    import json

    from ydbl.engine.results import Results

    img = np.zeros((100, 200, 3), dtype=np.uint8)
    data = torch.tensor([[10.0, 20.0, 60.0, 80.0, 0.9, 1.0], [150.0, 10.0, 190.0, 50.0, 0.5, 0.0]])
    r = Results(img, "a.jpg", {0: "cat", 1: "dog"}, boxes=data)
    assert len(r) == 2 and len(r[0]) == 1 and r[1].boxes.conf.item() == 0.5
    assert r.verbose() == "1 cat, 1 dog, "
    out = tmp_path / "labels" / "a.txt"
    r.save_txt(out, save_conf=True)
    lines = out.read_text().splitlines()
    assert lines[0] == "1 0.175 0.5 0.25 0.6 0.9"
    js = json.loads(r.to_json())
    assert js[0]["name"] == "dog" and js[1]["box"]["x2"] == 190.0
    assert list(r.to_df().columns) == ["name", "class", "confidence", "box"]
    r.update(boxes=torch.tensor([[-5.0, -5.0, 250.0, 120.0, 0.7, 0.0]]))
    assert r.boxes.xyxy.tolist() == [[0.0, 0.0, 200.0, 100.0]]
    pic = r.plot()
    assert pic.shape == img.shape and pic.dtype == np.uint8 and pic.any()
    # the box outline uses the palette colour of class 0 (#042AFF, BGR (255, 42, 4))
    assert tuple(pic[50, 0]) == (255, 42, 4)
    assert r.numpy().boxes.data.shape == (1, 6)
