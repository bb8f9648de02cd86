"""Multi-rank logic of the batch-sharded path on CPU (gloo, world size 2 and 3): shard bounds and
the all-gather that assembles per-image detections in global batch order."""

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


def _fake_dets(img: int, max_det: int):
    """Deterministic per-image detections so every rank can check the whole gathered batch."""
    n = (img * 7) % (max_det + 1)
    d = torch.zeros(max_det, 6)
    if n:
        d[:n] = torch.arange(n * 6, dtype=torch.float32).reshape(n, 6) + 1000 * img
    return d, n


def _worker(rank, world, port, B, max_det, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path

        sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "yolo-dbl_amd"))
        from ydbl.parallel import detections_list, gather_detections, shard_bounds

        s, e = shard_bounds(B, world, rank)
        det = torch.stack([_fake_dets(i, max_det)[0] for i in range(s, e)]) if e > s else torch.zeros(0, max_det, 6)
        cnt = torch.tensor([_fake_dets(i, max_det)[1] for i in range(s, e)], dtype=torch.int32)
        d_all, c_all = gather_detections(det, cnt, B)
        ok = d_all.shape == (B, max_det, 6)
        for i, di in enumerate(detections_list(d_all, c_all)):
            ref, n = _fake_dets(i, max_det)
            ok &= len(di) == n and torch.equal(di, ref[:n])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,B", [(2, 8), (2, 7), (3, 10)])
def test_gather_detections_gloo(world, B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, 5, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, True) for r in range(world)]
