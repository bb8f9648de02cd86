"""ydbl_nms alone on the bench's own candidates (DBL-n 640 bs32 fp16, synthetic blob images, trained-like
weights): per-image candidate counts and class mix, HIP-event time per launch for the class-split and
the one-workgroup-per-image forms, and (with the stamps build, scripts/build_stamps.sh detect, YDBL_LIB
pointing at it) the slowest workgroup's phase split.

    python scripts/nms_real.py [--stamps]

(build_dbg/ is listed in .gpurunignore; drop that line for a --stamps run on the GPU box.)
"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
ap = argparse.ArgumentParser()
ap.add_argument("--stamps", action="store_true")
ap.add_argument("--batch", type=int, default=32)
args = ap.parse_args()
if args.stamps:
    os.environ["YDBL_LIB"] = str(ROOT / "build_dbg" / "libydbl_stamps.so")
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CFGS  # noqa: E402
from ydbl import YOLO, _lib  # noqa: E402
from ydbl._lib import NmsDesc  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402

cfg, fx = CFGS["n"]
torch.manual_seed(0)  # as bench.py
model = YOLO(cfg, nc=3)
load_trained(model.model, ROOT / "tests" / "golden" / fx)
dev = torch.device("cuda", 0)
B = args.batch
sess = model.session(B, 640, 640, half=True, conf=0.25, iou=0.7, max_det=300, device=dev)
sess.load(blob_images(B, 640, seed=1234).to(dev))
for _ in range(3):
    sess()
torch.cuda.synchronize()
cnt = sess.cand_count.cpu().numpy()
cls = sess.cand_cls.cpu().numpy()
print("candidates per image:", cnt.tolist())
print("detections per image:", sess.count.cpu().tolist())
hist = np.zeros(3, dtype=int)
for b in range(B):
    hist += np.bincount(cls[b, : cnt[b]], minlength=3)[:3]
print("class mix of all candidates:", hist.tolist())
i = int(np.argmax(cnt))
print(f"largest image {i}: {cnt[i]} candidates, classes {np.bincount(cls[i, :cnt[i]], minlength=3).tolist()}")

cap = sess.cand_score.shape[1]
out = torch.zeros((B, 300, 6), device=dev)
oc = torch.zeros((B,), dtype=torch.int32, device=dev)
ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, cap, 30000)), dtype=torch.uint8, device=dev)  # zero-filled once (include/ydbl.h)
nd = NmsDesc(sess.cand_box.data_ptr(), sess.cand_score.data_ptr(), sess.cand_cls.data_ptr(), sess.cand_idx.data_ptr(),
             sess.cand_count.data_ptr(), B, cap, 0.7, 300, 30000, 0, 7680.0, 640.0, 640.0, out.data_ptr(),
             oc.data_ptr(), ws.data_ptr())
s = torch.cuda.current_stream().cuda_stream
for mode in ("1", "0"):
    os.environ["YDBL_NMS_GROUPS"] = mode
    _lib.check(_lib.lib.ydbl_nms(nd, s))
    torch.cuda.synchronize()
    same = torch.equal(out, sess.det) and torch.equal(oc, sess.count)
    torch.cuda._sleep(int(2e7))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        _lib.lib.ydbl_nms(nd, s)
    b.record()
    torch.cuda.synchronize()
    print(f"groups={mode}: {a.elapsed_time(b) / 20 * 1e3:.1f} us per ydbl_nms; equals the session's output: {same}")
    if args.stamps:
        buf = np.zeros(16 * 4096, dtype=np.uint64)
        assert _lib.lib.ydbl_nms_debug_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), len(buf)) == 0
        nwg = B * (8 if mode == "1" else 1)
        st = buf.reshape(-1, 16)[:nwg].astype(np.int64)
        d = (st[:, 1:4] - st[:, 0:3]) / 100.0
        tot = (st[:, 3] - st[:, 0]) / 100.0
        j = int(np.argmax(tot))
        print(f"  slowest wg {j}: sort {d[j,0]:.1f} stage {d[j,1]:.1f} sweep {d[j,2]:.1f} us ({st[j,5]} rounds, m={st[j,6]}); "
              f"a/b/c/d {st[j,7]/100:.1f}/{st[j,8]/100:.1f}/{st[j,9]/100:.1f}/{st[j,10]/100:.1f} us; "
              f"median wg {np.median(tot):.1f} us; start spread {(st[:,0].max()-st[:,0].min())/100:.1f} us; "
              f"pair-matrix path: rank words {(st[j,4]-st[j,2])/100:.1f} us, scan {(st[j,3]-st[j,4])/100:.1f} us")
