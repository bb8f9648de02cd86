"""Round 6: time ydbl_nms alone (HIP events over back-to-back launches): the rank-space pair-matrix path (images
<= 8192 candidates) against the sort + chunked sweep (YDBL_NMS_FAST=0, read per launch), per-image and class-split
schedules, on synthetic candidate sets shaped like the configs' worst images: DBL-s 640 bs4 sub-batch (1188
candidates), DBL-l 1280 bs4 (6210 of 33600 anchors), DBL-n bs16 (<= 645, the bench).

    python scripts/nms_wide_bench.py
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl import _lib  # noqa: E402
from ydbl._lib import NmsDesc, PredCandDesc  # noqa: E402


def pred(B, nc, A, counts, size, seed=0):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(B, 2, A, generator=g) * (size - 40) + 20
    wh = torch.rand(B, 2, A, generator=g) * (size / 8) + 4
    sc = torch.rand(B, nc, A, generator=g) * 0.2
    for b, k in enumerate(counts):  # k candidates above conf 0.25, classes dealt round-robin
        for c in range(nc):
            idx = torch.arange(c, k, nc)
            sc[b, c, idx] = 0.3 + 0.7 * torch.rand(len(idx), generator=g)
    m = A // 3  # clusters of overlapping boxes, as in tests/test_gpu_ops.py
    xy[:, :, 0: 3 * m: 3] = xy[:, :, 1: 3 * m: 3] + 1.5
    return torch.cat([xy, wh, sc], 1).cuda()


def run(counts, nc, A, size, per_image, reps=20):
    B = len(counts)
    p = pred(B, nc, A, counts, size).float().contiguous()
    dev = p.device
    cap = A
    cb = torch.empty((B, cap, 4), device=dev); cs = torch.empty((B, cap), device=dev)
    cc = torch.empty((B, cap), dtype=torch.int32, device=dev); ci = torch.empty((B, cap), dtype=torch.int32, device=dev)
    cn = torch.zeros((B,), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    pd = PredCandDesc(p.data_ptr(), B, nc, A, 0.25, 0, None, 0, cb.data_ptr(), cs.data_ptr(), cc.data_ptr(),
                      ci.data_ptr(), cn.data_ptr(), cap)
    _lib.check(_lib.lib.ydbl_pred_candidates(pd, s))
    res = {}
    for wide in ("1", "0"):
        os.environ["YDBL_NMS_FAST"] = wide
        out = torch.zeros((B, 300, 6), device=dev); cnt = torch.zeros((B,), dtype=torch.int32, device=dev)
        ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, cap, 30000)), dtype=torch.uint8, device=dev)
        nd = NmsDesc(cb.data_ptr(), cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(), B, cap, 0.7, 300,
                     30000, 0, 7680.0, float(size), float(size), out.data_ptr(), cnt.data_ptr(), ws.data_ptr(),
                     0, 0, per_image)
        _lib.check(_lib.lib.ydbl_nms(nd, s))
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(3):
            torch.cuda._sleep(int(1e7))
            a.record()
            for _ in range(reps):
                _lib.lib.ydbl_nms(nd, s)
            b.record()
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b) / reps * 1e3)
        res[wide] = (best, out.clone(), cnt.clone(), cn.tolist())
    os.environ.pop("YDBL_NMS_FAST")
    same = torch.equal(res["1"][1], res["0"][1]) and torch.equal(res["1"][2], res["0"][2])
    return res["1"][0], res["0"][0], same, res["1"][3], res["1"][2].tolist()


cases = [("DBL-s bs4: 1188,900,700,500", [1188, 900, 700, 500], 3, 8400, 640),
         ("4 x 1188", [1188] * 4, 3, 8400, 640),
         ("4 x 2500", [2500] * 4, 3, 8400, 640),
         ("DBL-l bs4: 6210,4000,3000,2000", [6210, 4000, 3000, 2000], 3, 33600, 1280),
         ("4 x 6210", [6210] * 4, 3, 33600, 1280),
         ("1 x 8192", [8192], 1, 33600, 1280),
         ("DBL-n bs16: 16 x 640", [640] * 16, 3, 8400, 640),
         # above 8192 candidates both columns run the select path (nms_select_sort): 3 buckets, and > max_nms 30000
         ("4 x 20000", [20000] * 4, 1, 33600, 1280),
         ("4 x 33600 (> max_nms)", [33600] * 4, 1, 33600, 1280)]
if len(sys.argv) > 1:  # one case under a profiler: python scripts/nms_wide_bench.py <case> <per_image> <wide>
    label, counts, nc, A, size = cases[int(sys.argv[1])]
    os.environ["YDBL_NMS_FAST"] = sys.argv[3]
    B = len(counts)
    p = pred(B, nc, A, counts, size).float().contiguous()
    cb = torch.empty((B, A, 4), device="cuda"); cs = torch.empty((B, A), device="cuda")
    cc = torch.empty((B, A), dtype=torch.int32, device="cuda"); ci = torch.empty((B, A), dtype=torch.int32, device="cuda")
    cn = torch.zeros((B,), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib.ydbl_pred_candidates(PredCandDesc(p.data_ptr(), B, nc, A, 0.25, 0, None, 0, cb.data_ptr(),
                                                          cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(),
                                                          A), s))
    out = torch.zeros((B, 300, 6), device="cuda"); cnt = torch.zeros((B,), dtype=torch.int32, device="cuda")
    ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, A, 30000)), dtype=torch.uint8, device="cuda")
    nd = NmsDesc(cb.data_ptr(), cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(), B, A, 0.7, 300, 30000, 0,
                 7680.0, float(size), float(size), out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), 0, 0,
                 int(sys.argv[2]))
    for _ in range(50):
        _lib.check(_lib.lib.ydbl_nms(nd, s))
    torch.cuda.synchronize()
    sys.exit(0)
for label, counts, nc, A, size in cases:
    for per_image in (1, 0):
        w, o, same, n, kept = run(counts, nc, A, size, per_image)
        print(f"{label:32s} per_image {per_image}: pair-matrix {w:7.1f} us   sort path {o:7.1f} us   bit-equal {same}   "
              f"cands {n}  kept {kept}", flush=True)
