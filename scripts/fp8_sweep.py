"""DBL-s 640 fp8 (BASELINE config 5): mAP50 drop vs the CPU oracle under the config-5 protocol
(tests/test_gpu_model.py::test_map50_config5_dbl_s_640) for a sweep of e4m3 MAC fractions."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-dbl_amd"), str(ROOT / "tests")]
import torch  # noqa: E402

import test_gpu_model as T  # noqa: E402
from oracle.ops import clip_boxes, non_max_suppression  # noqa: E402
from ydbl.utils.synthetic import blob_images  # noqa: E402

p, o = T._models("yolov13s_DBL.yaml", 3, ROOT / "tests" / "golden")
x = blob_images(16, 640, seed=1234)[[3, 13, 14, 15]]
with torch.no_grad():
    y, _ = o(x)
gt_conf = 0.0171
labels = []
for g in non_max_suppression(y, gt_conf, 0.7):
    clip_boxes(g[:, :4], (640, 640))
    labels.append(torch.cat([g[:, 5:6], g[:, :4]], 1))
batch = {"img": x, "cls": torch.cat([lb[:, 0] for lb in labels]), "bboxes": torch.cat([lb[:, 1:] for lb in labels]),
         "batch_idx": torch.cat([torch.full((len(lb),), i) for i, lb in enumerate(labels)])}
m_cpu = T._cpu_map50(o, x, labels, conf=gt_conf / 2)
for frac in (False, 0.25, 0.5, 0.75, 0.9, True):
    m = p.val(data=[batch], half=True, fp8=frac, conf=gt_conf / 2).box.map50
    print(f"fp8 fraction {frac}: mAP50 gpu {m:.4f} cpu {m_cpu:.4f} drop {m_cpu - m:+.4f}", flush=True)
