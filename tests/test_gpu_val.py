"""ydbl_match_predictions (device TP matrix) vs the oracle's box_iou + match_predictions
(U/models/yolo/detect/val.py:209-227, U/engine/validator.py:222-262): bit-exact per image."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _scene(n, max_det, nc, seed, empty_imgs=(), no_label_imgs=(), dup=False):
    """Random detections near random labels so every IoU band 0.5..0.95 is populated."""
    g = torch.Generator().manual_seed(seed)
    det = torch.zeros(n, max_det, 6)
    cnt = torch.zeros(n, dtype=torch.int32)
    boxes, cls, bidx = [], [], []
    for b in range(n):
        nl = 0 if b in no_label_imgs else int(torch.randint(1, 40, (1,), generator=g))
        xy = torch.rand(nl, 2, generator=g) * 500
        wh = torch.rand(nl, 2, generator=g) * 120 + 2
        gb = torch.cat([xy, xy + wh], 1)
        gc = torch.randint(0, nc, (nl,), generator=g).float()
        if dup and nl > 2:  # duplicated labels of another class: identical boxes, distinct classes
            gb[1] = gb[0]
            gc[1] = (gc[0] + 1) % nc
        boxes.append(gb); cls.append(gc); bidx.append(torch.full((nl,), b))
        k = 0 if b in empty_imgs else int(torch.randint(1, max_det + 1, (1,), generator=g))
        if k:
            src = torch.randint(0, max(nl, 1), (k,), generator=g)
            base = gb[src] if nl else torch.rand(k, 4, generator=g) * 300
            jit = (torch.rand(k, 4, generator=g) - 0.5) * 40 * torch.rand(k, 1, generator=g)
            pb = base + jit
            pb[:, 2:] = torch.maximum(pb[:, 2:], pb[:, :2] + 0.5)
            pc = gc[src] if nl else torch.zeros(k)
            flip = torch.rand(k, generator=g) < 0.2
            pc = torch.where(flip, torch.randint(0, nc, (k,), generator=g).float(), pc)
            conf = torch.sort(torch.rand(k, generator=g), descending=True).values
            det[b, :k] = torch.cat([pb, conf[:, None], pc[:, None]], 1)
            det[b, k:] = 7.0  # garbage past the count must be ignored
        cnt[b] = k
    return det, cnt, torch.cat(boxes), torch.cat(cls), torch.cat(bidx)


def _oracle(det, cnt, boxes, cls, bidx, iouv, single_cls=False):
    from oracle.metrics import box_iou, match_predictions

    out = torch.zeros(det.shape[0], det.shape[1], len(iouv), dtype=torch.bool)
    for b in range(det.shape[0]):
        p = det[b, : cnt[b]].clone()
        if single_cls:
            p[:, 5] = 0
        sel = bidx == b
        if len(p) and sel.any():
            out[b, : cnt[b]] = match_predictions(p[:, 5], cls[sel], box_iou(boxes[sel], p[:, :4]), iouv)
    return out


@pytest.mark.parametrize("n,max_det,nc,single,kw", [
    (4, 300, 3, False, {}),
    (3, 300, 80, False, {"empty_imgs": (1,), "no_label_imgs": (2,)}),
    (2, 600, 5, False, {"dup": True}),
    (5, 64, 3, True, {}),
    (1, 1000, 2, False, {}),
])
def test_match_bit_exact(n, max_det, nc, single, kw):
    from oracle.metrics import IOUV
    from ydbl.engine.validator import match_batch

    det, cnt, boxes, cls, bidx = _scene(n, max_det, nc, seed=n * 31 + max_det, **kw)
    # labels arrive interleaved across images: the launcher groups them stably
    perm = torch.randperm(len(bidx), generator=torch.Generator().manual_seed(5))
    ref = _oracle(det, cnt, boxes, cls, bidx, IOUV, single)
    got = match_batch(det.cuda(), cnt.cuda(), boxes[perm], cls[perm], bidx[perm], IOUV, single).cpu()
    # the permutation changes label order within an image only through the stable grouping, which
    # keeps each image's relative order of perm; re-derive the oracle on that order
    ref_p = _oracle(det, cnt, boxes[perm], cls[perm], bidx[perm], IOUV, single)
    assert torch.equal(got, ref_p)
    assert got.sum() > 0 and got.sum() < cnt.sum() * len(IOUV)
    # label order only matters on exact IoU ties, which random boxes do not produce
    assert torch.equal(got, ref)


def test_match_exact_ties_larger_label():
    """det0 has IoU exactly 0.6 with both labels: the reference's small-array argsort gives it the
    larger label index, leaving label 0 to det1 (tests/test_metrics.py pins the oracle on this)."""
    from oracle.metrics import IOUV
    from ydbl.engine.validator import match_batch

    boxes = torch.tensor([[0.0, 0.0, 10.0, 10.0], [5.0, 0.0, 15.0, 10.0]])
    cls = torch.tensor([1.0, 1.0])
    bidx = torch.tensor([0, 0])
    det = torch.zeros(1, 8, 6)
    det[0, 0] = torch.tensor([2.5, 0.0, 12.5, 10.0, 0.9, 1.0])
    det[0, 1] = torch.tensor([0.0, 0.0, 10.0, 10.0, 0.8, 1.0])
    cnt = torch.tensor([2], dtype=torch.int32)
    got = match_batch(det.cuda(), cnt.cuda(), boxes, cls, bidx, IOUV).cpu()
    ref = _oracle(det, cnt, boxes, cls, bidx, IOUV)
    assert torch.equal(got, ref)
    assert got[0, 0, :3].all() and not got[0, 0, 3:].any() and got[0, 1].all()


def test_match_no_labels_anywhere():
    from oracle.metrics import IOUV
    from ydbl.engine.validator import match_batch

    det, cnt, _, _, _ = _scene(2, 50, 3, seed=9, no_label_imgs=(0, 1))
    got = match_batch(det.cuda(), cnt.cuda(), torch.zeros(0, 4), torch.zeros(0), torch.zeros(0, dtype=torch.long),
                      IOUV)
    assert got.shape == (2, 50, 10) and not got.any()
