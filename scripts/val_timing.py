"""val() at conf 0.001 on DBL-l 1280 nc80: the validation setting is where candidate counts
are largest (multi-label, every class score above 0.001), so it is the NMS path's stress case.

Weights: the DBL-l trained-like fixture (tests/golden, nc3) for every tensor whose shape matches; the nc80 class
1x1 weights and biases are the fixture's three class rows tiled over the 80 classes, each row scaled by
1 + 0.05 N(0,1) (seed 0) so that the classes' scores differ.
Images: synthetic blob images; pseudo ground truth = the same model's conf-0.25 detections.  Prints candidates per
image, the val() wall time per image (fp16, rect tensor batches, bs 8 -> two bs4 sessions is NOT used: val runs one
session per batch shape, streams 1), the session call alone (HIP events) and ydbl_nms alone on its candidates.

    python scripts/val_timing.py [--batch 8] [--images 16]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CFGS  # noqa: E402
from ydbl import YOLO, _lib  # noqa: E402
from ydbl._lib import NmsDesc  # noqa: E402
from ydbl.utils.synthetic import blob_images  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--images", type=int, default=16)
ap.add_argument("--imgsz", type=int, default=1280)
args = ap.parse_args()

cfg, fx = CFGS["l"]
torch.manual_seed(0)
model = YOLO(cfg, nc=80)
sd = model.model.state_dict()
tiled = set()
g = torch.Generator().manual_seed(0)
with np.load(str(ROOT / "tests" / "golden" / fx), allow_pickle=False) as z:
    for k in z.files:
        v = torch.from_numpy(z[k])
        if v.numel() == sd[k].numel():
            sd[k].copy_(v.view_as(sd[k]))
        elif v.dim() and v.shape[0] == 3 and sd[k].shape[0] == 80 and v[0].numel() == sd[k][0].numel():  # class rows
            rows = v.reshape(3, -1).repeat(27, 1)[:80]
            sd[k].copy_((rows * (1 + 0.05 * torch.randn(80, 1, generator=g))).view_as(sd[k]))
            tiled.add(k)
# the class 1x1 weights are not in the fixture (random init): tile their first 3 rows the same way
for k, t in sd.items():
    if k not in tiled and k.endswith("weight") and t.dim() == 4 and t.shape[0] == 80 and t.shape[2:] == (1, 1):
        t.copy_(t[:3].repeat(27, 1, 1, 1)[:80] * (1 + 0.05 * torch.randn(80, 1, 1, 1, generator=g)))
        tiled.add(k)
print(f"fixture applied; {len(tiled)} class tensors tiled to 80 classes")
dev = torch.device("cuda", 0)
B, S, N = args.batch, args.imgsz, args.images
x = blob_images(N, S, seed=1234)

# pseudo ground truth from the model's own conf-0.25 detections
gt = model.session(B, S, S, half=True, conf=0.25, iou=0.7, max_det=300, device=dev)
labels = []
for i in range(0, N, B):
    det, cnt = gt(x[i:i + B].to(dev))
    det, cnt = det.cpu(), cnt.cpu()
    for j in range(len(cnt)):
        d = det[j, : int(cnt[j])]
        labels.append(torch.cat([d[:, 5:6], d[:, :4]], 1))
batches = []
for i in range(0, N, B):
    lb = labels[i:i + B]
    batches.append({"img": x[i:i + B], "cls": torch.cat([l[:, 0] for l in lb]), "bboxes": torch.cat([l[:, 1:] for l in lb]),
                    "batch_idx": torch.cat([torch.full((len(l),), k) for k, l in enumerate(lb)])})
print(f"pseudo ground truth: {sum(len(l) for l in labels)} boxes over {N} images")

m = model.val(data=batches, half=True, batch=B)  # compile + warm
torch.cuda.synchronize()
reps = 3
t0 = time.perf_counter()
for _ in range(reps):
    m = model.val(data=batches, half=True, batch=B)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps
print(f"val(): {wall * 1e3:.1f} ms for {N} images = {wall * 1e3 / N:.2f} ms per image "
      f"({N / wall:.1f} img/s, host metrics included); mAP50 vs pseudo GT {m.box.map50:.3f}")

sess = model.session(B, S, S, half=True, conf=0.001, iou=0.7, max_det=300, multi_label=True, device=dev, clip=True)
xb = x[:B].to(dev)
sess(xb)
torch.cuda.synchronize()
cnt = sess.cand_count.cpu().numpy()
print(f"candidates per image (conf 0.001, multi-label): {cnt.tolist()} (cap {sess.cand_score.shape[1]}); "
      f"detections {sess.count.cpu().tolist()}")
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
sess.load(xb)
a.record()
for _ in range(10):
    sess()
b.record()
torch.cuda.synchronize()
print(f"session call (forward + decode + NMS, bs{B}, one graph): {a.elapsed_time(b) / 10:.2f} ms")

cap = sess.cand_score.shape[1]
out = torch.zeros((B, 300, 6), device=dev)
oc = torch.zeros((B,), dtype=torch.int32, device=dev)
ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, cap, 30000)), dtype=torch.uint8, device=dev)
nd = NmsDesc(sess.cand_box.data_ptr(), sess.cand_score.data_ptr(), sess.cand_cls.data_ptr(), sess.cand_idx.data_ptr(),
             sess.cand_count.data_ptr(), B, cap, 0.7, 300, 30000, 0, 7680.0, float(S), float(S), out.data_ptr(),
             oc.data_ptr(), ws.data_ptr())
s = torch.cuda.current_stream().cuda_stream
_lib.check(_lib.lib.ydbl_nms(nd, s))
torch.cuda.synchronize()
same = torch.equal(out, sess.det) and torch.equal(oc, sess.count)
a.record()
for _ in range(20):
    _lib.lib.ydbl_nms(nd, s)
b.record()
torch.cuda.synchronize()
print(f"ydbl_nms alone on these candidates: {a.elapsed_time(b) / 20 * 1e3:.1f} us per bs{B} call; "
      f"equals the session's output: {same}")
