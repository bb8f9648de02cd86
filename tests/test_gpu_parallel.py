"""The batch-sharded path at world size 2 WITH the GPU sessions (ydbl.parallel.ShardedPredictor): two processes
share the box's one MI355X over a gloo group (the records pass through host memory there; on an 8-GPU node the
same code runs one rank per GPU over RCCL).  Global batch 5 -> slices of 3 and 2 images, so the last rank carries
a padding row.  Each rank's rows of the gathered global result equal its own session's output bit for bit,
rank 0 recomputes rank 1's slice with a session of the same batch (the gathered rows equal it bit for bit), and
rank 0 checks every gathered row against the oracle under the fp16 rule of tests/test_gpu_e2e.py: final
detections matched both ways against the oracle's fp64 answer, with no more mismatches than twice the oracle's own
half-precision leg + 2 and no more borderline decisions than twice that leg's + 3."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path

        root = Path(__file__).resolve().parent.parent
        sys.path[:0] = [str(root / "yolo-dbl_amd"), str(root)]
        from ydbl import YOLO
        from ydbl.parallel import ShardedPredictor, shard_bounds
        from ydbl.utils.synthetic import blob_images, load_trained

        torch.manual_seed(0)
        m = YOLO("yolov13n_DBL.yaml", nc=3)
        load_trained(m.model, root / "tests" / "golden" / "trained_yolov13n_DBL_nc3.npz")
        B = 5
        x = blob_images(B, 160, seed=21).cuda()
        sp = ShardedPredictor(m, B, 160, 160, "cuda:0", half=True, conf=0.05, iou=0.7)
        det_all, cnt_all = sp(images_global=x)
        torch.cuda.synchronize()
        s, e = shard_bounds(B, world, rank)
        own_d, own_c = sp.session.det, sp.session.count
        ok = torch.equal(det_all[s:e], own_d) and torch.equal(cnt_all[s:e], own_c)
        if rank == 0:  # rank 1's slice recomputed here with a session of its batch
            s1, e1 = shard_bounds(B, world, 1)
            ref = m.session(e1 - s1, 160, 160, half=True, conf=0.05, iou=0.7, streams=1)
            d1, c1 = ref(x[s1:e1])
            torch.cuda.synchronize()
            ok = ok and torch.equal(det_all[s1:e1], d1) and torch.equal(cnt_all[s1:e1], c1)
            ok = ok and int(cnt_all.sum()) > 0
            # the gathered global result against the oracle (not only against the sessions that produced it)
            sys.path.insert(0, str(root / "tests"))
            from parity_util import detections, err_stats, fp16_rule, match_detections, oracle_legs, oracle_only

            o = oracle_only("n", 3, root / "tests" / "golden")
            with torch.no_grad():
                ys, _ = oracle_legs(o, x.cpu(), ("fp64", "fp16"))
            y64 = ys["fp64"]
            st16 = err_stats(ys["fp16"], y64)
            tb, tc = fp16_rule(st16)
            ref_dets = detections(y64, 0.05, 0.7, (160, 160))
            m16 = match_detections(ref_dets, detections(ys["fp16"], 0.05, 0.7, (160, 160)), y64, 0.05, 0.7, tb, tc)
            got = [det_all[i, : int(cnt_all[i])].cpu() for i in range(B)]
            mg = match_detections(ref_dets, got, y64, 0.05, 0.7, tb, tc)
            print(f"world 2 gathered vs oracle fp64: {mg['pairs']} pairs, {mg['borderline']} borderline, "
                  f"{len(mg['mismatches'])} mismatches (oracle half leg: {m16['borderline']} / {len(m16['mismatches'])})",
                  flush=True)
            ok = (ok and mg["pairs"] > 0 and len(mg["mismatches"]) <= 2 * len(m16["mismatches"]) + 2
                  and mg["borderline"] <= 2 * m16["borderline"] + 3)
        q.put((rank, bool(ok), [int(c) for c in cnt_all.tolist()]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_sharded_predictor_world2_gpu_sessions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    got.sort()
    assert [g[1] for g in got] == [True, True], got
    assert got[0][2] == got[1][2]  # both ranks hold the same global counts
