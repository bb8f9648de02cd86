"""Generate the end-to-end parity fixtures tests/golden/e2e_<model><size>.npz (run in the CPU container).

For each BASELINE model/size (DBL-n 640, DBL-s 640, DBL-l(DBL2) 1280, and DBL-x(DBL2) 640) the oracle restatement
(oracle/model.py; nothing from the reference is run) evaluates the first reference images of the
synthetic batch blob_images(B_full, S, seed=1234) on the trained-like state_dict fixture in three
precisions.  Stored:
- ``y64``: fp64 answer of the BN-folded network [R, 4+nc, A], saved as fp32 (rounding <= 1e-4 px);
- ``d32``: the reference path's own fp32 answer minus y64, as fp16 (|d32| <= ~1e-2 px, so the stored
  difference is exact to ~1e-5 px): the tests report the GPU's direct distance from the oracle's fp32 leg;
- ``meta``: JSON with the batch spec, the predict conf used by the tests, and the deviation of the
  reference path's own fp32 and fp16 legs from y64 (max and p99.9 of boxes/scores, and the
  final-detection mismatch count under the test's rule).  The GPU tests (tests/test_gpu_e2e.py) bound the
  GPU's deviations by these times a per-fixture factor (tests/parity_util.py FP32_FACTOR: 2, 2.5 on the DBL-s
  max; fp16: 2) and its direct distance from the fp32 leg by 3x its deviation.

Usage: python tests/golden/make_e2e.py
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "yolo-dbl_amd")]

from parity_util import (detections, err_stats, fp16_rule, fp32_rule, match_detections,  # noqa: E402
                         oracle_only, oracle_legs)
from ydbl.utils.synthetic import blob_images  # noqa: E402

OUT = Path(__file__).resolve().parent
# Reference images: the first and last image of each bs/2 sub-batch graph of the bench layout (streams=2: images
# 15 and 16 sit on either side of the split, 31 is the batch tail, where the flattened-pixel kernels put their
# ragged last tile) plus image 1; l1280 bs8: the first and the last image.
CASES = {"n640": ("n", 640, 32, [0, 1, 15, 16, 31]), "s640": ("s", 640, 32, [0, 1, 15, 16, 31]),
         "l1280": ("l", 1280, 8, [0, 7]), "x640": ("x", 640, 8, [0, 1])}


def choose_conf(y64):
    """The predict default 0.25 when it keeps >= 20 detections on the reference images, else the
    99.5th percentile of the best-class scores (the untrained-like DBL-s fixture scores below 0.1)."""
    if sum(len(d) for d in detections(y64, 0.25, 0.7, (1, 1))) >= 20:
        return 0.25
    sc = y64[:, 4:].amax(1).flatten().float()
    return float(f"{torch.quantile(sc, 0.995).item():.3g}")


def main(names=None):
    for name, (scale, S, B, ref) in CASES.items():
        if names and name not in names:
            continue
        o = oracle_only(scale, 3, OUT)
        x = blob_images(B, S, seed=1234)[ref]
        ys, secs = oracle_legs(o, x, ("fp64", "fp32", "fp16"))
        y64 = ys["fp64"]
        conf = choose_conf(y64)
        meta = {"scale": scale, "imgsz": S, "batch_full": B, "seed": 1234, "ref_images": ref, "nc": 3,
                "conf": conf, "iou": 0.7, "x_sum": float(x.double().sum())}
        ref_dets = detections(y64, conf, 0.7, (S, S))
        meta["ref_dets"] = [len(d) for d in ref_dets]
        for leg, rule in (("fp32", fp32_rule), ("fp16", fp16_rule)):
            st = err_stats(ys[leg], y64)
            tb, tc = rule(st)
            m = match_detections(ref_dets, detections(ys[leg], conf, 0.7, (S, S)), y64, conf, 0.7, tb, tc)
            st.update({"det_mismatches": len(m["mismatches"]), "det_borderline": m["borderline"],
                       "det_pairs": m["pairs"], "det_box_dev": m["box_dev"], "det_conf_dev": m["conf_dev"]})
            meta[f"oracle_{leg}"] = st
        d32 = (ys["fp32"].double() - y64).half().numpy()
        np.savez_compressed(OUT / f"e2e_{name}.npz", y64=y64.float().numpy(), d32=d32, meta=np.array(json.dumps(meta)))
        print(name, {k: round(v, 2) for k, v in secs.items()}, json.dumps(meta))


if __name__ == "__main__":
    main(sys.argv[1:])
