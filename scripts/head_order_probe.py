"""The Detect head's per-level launches in a different order on the two sub-batch branches (DBL-n bs32 fp16,
streams=2): the levels are independent until the decode, so branch 1 can run P5 -> P4 -> P3 while branch 0 runs
P3 -> P4 -> P5, pairing one branch's full-chip P3 kernels with the other's latency-bound P5 ones instead of running
the same level on both at once.  Captures both layouts as one-graph branch pairs and times them alternately.

    python scripts/head_order_probe.py
"""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

from branch_offset_probe import run_steps  # noqa: E402
from ydbl import YOLO  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402


def level_groups(steps):
    """Index ranges of the head's per-level launch groups: each level starts at a 'Detect.box3' launch or, for the
    unfused P5 box branch, at the first of its two Conv3x3 launches; the head ends at the decode."""
    dec = next(i for i, st in enumerate(steps) if st.what == "Detect.decode")
    first = next(i for i, st in enumerate(steps) if st.what == "Detect.box3")
    starts = [i for i in range(first, dec) if steps[i].what == "Detect.box3"]
    # the P5 level: after the last box3 group's three launches
    starts.append(starts[-1] + 3)
    bounds = starts + [dec]
    return [(bounds[k], bounds[k + 1]) for k in range(len(starts))], dec


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = YOLO("yolov13n_DBL.yaml", nc=3)
    load_trained(model.model, ROOT / "tests" / "golden" / "trained_yolov13n_DBL_nc3.npz")
    sess = model.session(32, 640, 640, half=True, conf=0.25, iou=0.7, max_det=300, device=dev, streams=2)
    sess.load(blob_images(32, 640, seed=1234).to(dev))
    sess.launch()
    torch.cuda.synchronize(dev)
    ref = (sess.det.clone(), sess.count.clone())
    p0, p1 = sess.plans
    groups, dec = level_groups(p1.steps)
    print("head level groups:", [[p1.steps[i].what for i in range(a, b)] for a, b in groups], flush=True)
    first = groups[0][0]
    rev = p1.steps[:first] + [st for a, b in reversed(groups) for st in p1.steps[a:b]] + p1.steps[dec:]
    assert len(rev) == len(p1.steps)

    def capture(steps1):
        side = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cap = torch.cuda.current_stream(dev)
            side.wait_stream(cap)
            run_steps(p0, p0.steps, cap.cuda_stream)
            with torch.cuda.stream(side):
                run_steps(p1, steps1, side.cuda_stream)
            cap.wait_stream(side)
        torch.cuda.synchronize(dev)
        return g

    g_same, g_rev = capture(p1.steps), capture(rev)
    g_rev.replay()
    torch.cuda.synchronize(dev)
    assert torch.equal(sess.det, ref[0]) and torch.equal(sess.count, ref[1]), "reordered head changed the output"

    def t(g, n=40):
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n * 1e3

    a, b = [], []
    for _ in range(5):
        a.append(t(g_same))
        b.append(t(g_rev))
    a.sort()
    b.sort()
    print(f"same head order on both branches: median {a[2]:.4f} ms/step ({32 / a[2] * 1e3:.0f} img/s)", flush=True)
    print(f"branch 1 head reversed (P5 first): median {b[2]:.4f} ms/step ({32 / b[2] * 1e3:.0f} img/s)  "
          f"({100 * (a[2] / b[2] - 1):+.2f} %)", flush=True)


if __name__ == "__main__":
    main()
