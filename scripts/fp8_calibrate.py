"""Record the fp8 (BASELINE config 5) calibration of the DBL-s fixture weights and measure its mAP50 drop per share.

Calibration set: blob_images(32, 640, seed=4321) -- disjoint from the evaluation images (seed 1234) -- run through
one bs32 fp16 plan: per-conv activation scales and bias corrections taken at each conv's launch, and the
per-conv sensitivity ranking (ydbl.quant.calibrate).  Saved as tests/golden/fp8_calib_yolov13s_DBL_nc3.json, which
bench.py --fp8 and the config-5 tests load, so "25 %" names ONE layer set and one set of scales whatever batch or
sub-batch layout runs it.  Then the config-5 protocol (tests/test_gpu_model.py::test_map50_config5_dbl_s_640: the
16 evaluation images, pseudo-GT = the CPU oracle's fp32 detections at conf 0.0171, val at conf 0.001) for each share,
twice (the drop must repeat exactly).

    python scripts/fp8_calibrate.py [--no-save] [--head-metric] [share ...]     (default shares: 0.1 0.25 0.5 1.0)

Ranking: each candidate conv ALONE in e4m3, the mean |delta| of the Detect head maps (ydbl.quant.calibrate).  Layer
sets (default): greedy over that order on the calibration images, a conv kept only if the kept set's mAP50 drop
against the fp16 path's own detections there grows by <= TAU (product code only: no oracle); --head-metric: the
ranking's MAC-budget sets (select_by_mac_budget) instead.
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-dbl_amd"), str(ROOT / "tests")]
import torch  # noqa: E402

import test_gpu_model as T  # noqa: E402
from oracle.ops import clip_boxes, non_max_suppression  # noqa: E402
from ydbl import quant  # noqa: E402
from ydbl.utils.synthetic import blob_images  # noqa: E402

CAL = ROOT / "tests" / "golden" / "fp8_calib_yolov13s_DBL_nc3.json"
SHARES = (0.1, 0.25)  # the shares recorded as explicit greedy sets (1.0 = every candidate)
TAU = 0.005  # largest mAP50-drop increase on the calibration images a kept conv may add


def main():
    args = sys.argv[1:]
    save = "--no-save" not in args
    shares = [float(a) for a in args if not a.startswith("--")] or [0.1, 0.25, 1.0]
    p, o = T._models("yolov13s_DBL.yaml", 3, ROOT / "tests" / "golden")
    greedy = "--head-metric" not in args
    if save or not CAL.exists():
        xc = blob_images(32, 640, seed=4321)
        s = p.session(32, 640, 640, half=True, conf=0.25, iou=0.7, keep_pred=True, use_graph=False)
        s.load(xc.cuda())
        cal = quant.calibrate([s.plan], s.plan.run, head=s.compiled.feats, rank=True, meta={
            "model": "yolov13s_DBL.yaml nc 3", "weights": "tests/golden/trained_yolov13s_DBL_nc3.npz",
            "calibration_images": "ydbl.utils.synthetic.blob_images(32, 640, seed=4321), one bs32 fp16 plan",
            "sens": "mean |delta| of the Detect head maps with the conv alone in e4m3",
            "sets": ("greedy on the calibration images: candidates in sens order, each kept only if the mAP50 drop of "
                     "the kept set (against the fp16 path's own detections at conf .25, val protocol) grows by <= "
                     f"{TAU}; the set of a share = the kept convs within its MAC budget") if greedy else "none",
            "script": "scripts/fp8_calibrate.py"})
        p._sessions.clear()
        if greedy:
            s16 = p.session(32, 640, 640, half=True, conf=0.25, iou=0.7)
            d, c = s16(xc.cuda())
            torch.cuda.synchronize()
            cnt = c.cpu().tolist()
            dets = [d[i, : cnt[i]].cpu() for i in range(32)]
            cb = {"img": xc, "cls": torch.cat([t[:, 5] for t in dets]), "bboxes": torch.cat([t[:, :4] for t in dets]),
                  "batch_idx": torch.cat([torch.full((len(t),), i) for i, t in enumerate(dets)])}
            p._sessions.clear()
            base = p.val(data=[cb], half=True, conf=0.001).box.map50
            total = sum(cal.macs.values())

            def drop(keys):
                sub = quant.Fp8Calibration({k: cal.qs[k] for k in keys}, {k: cal.delta[k] for k in keys},
                                           macs={k: cal.macs[k] for k in keys})
                p._sessions.clear()
                return base - p.val(data=[cb], half=True, conf=0.001, fp8=True, fp8_calibration=sub).box.map50

            kept, cur, macs = [], 0.0, 0
            for k in sorted(cal.sens, key=lambda k: (cal.sens[k], k)):
                if (macs + cal.macs[k]) / total > max(SHARES) + 1e-9:
                    continue
                d_k = drop(kept + [k])
                ok = d_k - cur <= TAU
                print(f"   greedy {k:24s} drop {d_k:+.4f} ({'kept' if ok else 'skipped'}), MAC share "
                      f"{(macs + cal.macs[k] * ok) / total:.3f}", flush=True)
                if ok:
                    kept.append(k)
                    cur, macs = d_k, macs + cal.macs[k]
                    for sh in SHARES:  # the set of a share: the kept convs while within its budget
                        if macs / total <= sh + 1e-9:
                            cal.sets[f"{sh:g}"] = sorted(kept)
            # a share the low-drop pass did not fill: forward selection -- add the candidate whose addition moves the
            # calibration drop least, until the next would pass the share's MAC budget
            for sh in SHARES:
                if cal.sets.get(f"{sh:g}") is not None and macs / total >= sh - 0.02:
                    continue
                while True:
                    left = [k for k in cal.qs if k not in kept and (macs + cal.macs[k]) / total <= sh + 1e-9]
                    if not left:
                        break
                    trials = {k: drop(kept + [k]) for k in left}
                    k = min(trials, key=lambda k: (trials[k], k))
                    kept.append(k)
                    cur, macs = trials[k], macs + cal.macs[k]
                    print(f"   forward {k:24s} drop {cur:+.4f}, MAC share {macs / total:.3f}", flush=True)
                cal.sets[f"{sh:g}"] = sorted(kept)
            p._sessions.clear()
        cal.save(CAL)
        print(f"saved {CAL.relative_to(ROOT)}: {len(cal.qs)} candidate convs", flush=True)
    cal = quant.Fp8Calibration.load(CAL)
    for k in sorted(cal.sens, key=cal.sens.get):
        print(f"   {k:28s} sens {cal.sens[k]:.4g}  MAC share {cal.macs[k] / sum(cal.macs.values()):.4f}")
    x = blob_images(16, 640, seed=1234)
    with torch.no_grad():
        y, _ = o(x)
    labels = []
    for g in non_max_suppression(y, 0.0171, 0.7):
        clip_boxes(g[:, :4], (640, 640))
        labels.append(torch.cat([g[:, 5:6], g[:, :4]], 1))
    batch = {"img": x, "cls": torch.cat([lb[:, 0] for lb in labels]),
             "bboxes": torch.cat([lb[:, 1:] for lb in labels]),
             "batch_idx": torch.cat([torch.full((len(lb),), i) for i, lb in enumerate(labels)])}
    m_cpu = T._cpu_map50(o, x, labels, conf=0.001)
    m16 = p.val(data=[batch], half=True, conf=0.001).box.map50
    print(f"fp16: mAP50 gpu {m16:.4f} cpu {m_cpu:.4f} drop {m_cpu - m16:+.4f}", flush=True)
    for share in shares:
        keys = cal.switched(share)
        drops = []
        for _ in range(2):
            p._sessions.clear()
            m = p.val(data=[batch], half=True, fp8=True if share >= 1 else share, conf=0.001,
                      fp8_calibration=str(CAL)).box.map50
            drops.append(m_cpu - m)
        print(f"share {share}: {len(keys)} convs, MAC fraction {cal.mac_fraction(keys):.4f}, mAP50 drop "
              f"{drops[0]:+.4f} / {drops[1]:+.4f} (two runs); layers {keys}", flush=True)


if __name__ == "__main__":
    main()
