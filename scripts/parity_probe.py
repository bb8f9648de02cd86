"""Measure end-to-end deviations at the BASELINE shapes: GPU (fp32/fp16/fp8) and oracle (fp32/fp16) vs the
oracle's fp64 answer, plus final-detection agreement.  Used to set the tolerances written in
tests/test_gpu_e2e.py.  Writes gpurun_out/parity_probe.jsonl."""

import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "yolo-dbl_amd")]

from parity_util import build_pair, class_agreement, detections, err_stats, gpu_pred, oracle_legs  # noqa: E402
from ydbl.utils.synthetic import blob_images  # noqa: E402

G = ROOT / "tests" / "golden"
OUT = ROOT / "gpurun_out" / "parity_probe.jsonl"
OUT.parent.mkdir(exist_ok=True)


def log(d):
    print(json.dumps(d), flush=True)
    with OUT.open("a") as f:
        f.write(json.dumps(d) + "\n")


def nearest_dev(ref, got):
    """per ref det: min over same-class got dets of max |box| dev; returns sorted list."""
    devs = []
    for r, g in zip(ref, got):
        for d in r:
            if len(g):
                same = g[:, 5] == d[5]
                dv = torch.where(same, (g[:, :4] - d[:4]).abs().amax(1), torch.full((len(g),), 1e9))
                devs.append(dv.min().item())
            else:
                devs.append(1e9)
    devs.sort()
    return devs


for scale, B, S, modes in [("n", 2, 640, ("fp32", "fp16", "fp8")), ("s", 2, 640, ("fp32", "fp16", "fp8")),
                           ("l", 1, 1280, ("fp32", "fp16"))]:
    p, o = build_pair(scale, 3, G)
    x = blob_images(B, S, seed=1234)
    t0 = time.time()
    ys, secs = oracle_legs(o, x, ("fp64", "fp32", "fp16"))
    y64 = ys["fp64"]
    rec = {"cfg": f"{scale}{S} bs{B}", "oracle_secs": secs}
    for leg in ("fp32", "fp16"):
        rec[f"oracle_{leg}"] = err_stats(ys[leg], y64)
    ref_dets = detections(y64, 0.25, 0.7, (S, S))
    o32_dets = detections(ys["fp32"], 0.25, 0.7, (S, S))
    rec["n_ref_dets"] = sum(len(d) for d in ref_dets)
    rec["oracle_fp32_det_devs_tail"] = nearest_dev(ref_dets, o32_dets)[-5:]
    for mode in modes:
        t1 = time.time()
        yg, dg = gpu_pred(p, x, half=mode != "fp32", fp8=mode == "fp8", calib=blob_images(B, S, seed=4321))
        st = err_stats(yg, y64)
        st["gpu_secs"] = round(time.time() - t1, 2)
        st["class_agree"] = class_agreement(yg, y64, 2 * st["conf_max"])
        st["n_dets"] = sum(len(d) for d in dg)
        st["det_devs_tail"] = nearest_dev(ref_dets, dg)[-5:]
        st["det_devs_rev_tail"] = nearest_dev(dg, ref_dets)[-5:]
        rec[f"gpu_{mode}"] = st
    log(rec)
