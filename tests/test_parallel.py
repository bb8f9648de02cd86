"""Multi-rank logic of the batch-sharded path on CPU (gloo, world size 2 and 3): shard bounds and the one
all-gather of per-image records that assembles the detections in global batch order.  Each rank's records
hold real detections: the oracle's (CPU restatement of the reference path) on that rank's slice of a
seeded DBL-n 128x128 batch, max_det 20 so full and empty rows both occur."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_shard_bounds_cover_batch():
    from ydbl.parallel import shard_bounds

    for B in (1, 7, 32, 33, 64):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(B, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(8, 2, 2)


def _oracle_shard_dets(m, x, s, e, max_det):
    """The reference path's detections (oracle: fused DBL-n fp32 forward + NMS, U/utils/ops.py:167-316) of
    images [s, e) of x, computed as one batch -- what rank r's GPU session computes for its slice."""
    from oracle.ops import non_max_suppression

    if e <= s:
        return []
    with torch.inference_mode():
        y, _ = m(x[s:e])
    return non_max_suppression(y, 0.05, 0.7, max_det=max_det)


def _worker(rank, world, port, B, max_det, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path

        root = Path(__file__).resolve().parent.parent
        sys.path[:0] = [str(root / "yolo-dbl_amd"), str(root)]
        from oracle.model import build_model
        from ydbl.parallel import detections_list, gather_detections, record_views, record_width, shard_bounds
        from ydbl.utils.synthetic import blob_images, load_trained

        torch.manual_seed(0)
        m = build_model("yolov13n_DBL.yaml", nc=3)
        load_trained(m, root / "tests" / "golden" / "trained_yolov13n_DBL_nc3.npz")
        m.fuse()
        x = blob_images(B, 128, seed=7)
        s, e = shard_bounds(B, world, rank)
        b_max = -(-B // world)
        # this rank's record buffer, filled the way ydbl_nms fills it (rows past the count zero, padding rows empty)
        rec = torch.zeros(b_max, record_width(max_det))
        det, cnt = record_views(rec, max_det)
        for i, d in enumerate(_oracle_shard_dets(m, x, s, e, max_det)):
            det[i, : len(d)] = d
            cnt[i] = len(d)
        d_all, c_all = gather_detections(rec, B, max_det)
        ok = d_all.shape == (B, max_det, 6) and c_all.shape == (B,)
        ref = [d for r in range(world) for d in _oracle_shard_dets(m, x, *shard_bounds(B, world, r), max_det)]
        got = detections_list(d_all, c_all)
        ok &= len(got) == B and sum(len(d) for d in ref) > 0
        for di, ri in zip(got, ref):
            ok &= torch.equal(di, ri)
        ok &= bool((d_all[c_all.long() == 0] == 0).all())
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,B", [(2, 8), (3, 10)])  # even, and ragged (last rank one image short)
def test_gather_records_gloo(world, B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, 20, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, True) for r in range(world)]


def test_record_views_layout():
    from ydbl.parallel import record_views, record_width

    assert record_width(300) == 1804 and record_width(1) == 8
    rec = torch.zeros(3, record_width(4))
    det, cnt = record_views(rec, 4)
    assert det.shape == (3, 4, 6) and cnt.shape == (3,) and cnt.dtype == torch.int32
    det[1, 2, 5] = 7.0
    cnt[2] = 3
    assert rec[1, 2 * 6 + 5] == 7.0 and rec[2].view(torch.int32)[24] == 3
    assert det.stride(0) == cnt.stride(0) == record_width(4)
    with pytest.raises(ValueError):
        record_views(torch.zeros(2, 30), 4)
