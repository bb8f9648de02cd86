"""Is the high-resolution prefix of DBL-n cheaper as ONE bs32 pass or as the bench's two concurrent bs16 branches?
Captures, for each prefix length K (the first K launches of the plan), a graph of the bs32 single-stream plan's
first K launches and a graph of the two bs16 sub-batch plans' first K launches as concurrent branches, and times
both (replays alternating, several rounds).  A prefix that is cheaper at bs32 could run as one pass before the
graph forks into the two sub-batch branches.

    python scripts/split_prefix_probe.py [K ...]            (bs32 pass vs 2 branches)
    python scripts/split_prefix_probe.py --s4 [K ...]       (2 bs16 branches vs 4 bs8 branches)
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


def main():
    s4 = "--s4" in sys.argv
    ks = [int(a) for a in sys.argv[1:] if a != "--s4"] or [1, 2, 5, 9, 10, 12, 28]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = YOLO("yolov13n_DBL.yaml", nc=3)
    load_trained(model.model, ROOT / "tests" / "golden" / "trained_yolov13n_DBL_nc3.npz")
    kw = dict(half=True, conf=0.25, iou=0.7, max_det=300, device=dev)
    s2 = model.session(32, 640, 640, streams=2, **kw)
    s1 = model.session(32, 640, 640, streams=4 if s4 else 1, **kw)
    x = blob_images(32, 640, seed=1234).to(dev)
    s2.load(x)
    s1.load(x)
    for _ in range(2):
        s2.launch()
        s1.launch()
    torch.cuda.synchronize(dev)
    p1, p2 = s1.plan, s2.plans
    p4 = s1.plans if s4 else None
    print("launches:", ", ".join(f"{i}:{st.what}" for i, st in enumerate(p1.steps[:30])), flush=True)

    def single(k):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run_steps(p1, p1.steps[:k], torch.cuda.current_stream(dev).cuda_stream)
        return g

    def branches(k, plans=None):
        plans = plans or p2
        sides = [torch.cuda.Stream(dev) for _ in plans[1:]]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cap = torch.cuda.current_stream(dev)
            for side in sides:
                side.wait_stream(cap)
            run_steps(plans[0], plans[0].steps[:k], cap.cuda_stream)
            for pl, side in zip(plans[1:], sides):
                with torch.cuda.stream(side):
                    run_steps(pl, pl.steps[:k], side.cuda_stream)
            for side in sides:
                cap.wait_stream(side)
        return g

    def t(g, n=40):
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n * 1e6

    for k in [min(k, len(p1.steps)) for k in ks]:
        gs, gb = (branches(k, p4) if s4 else single(k)), branches(k)
        a, b = [], []
        for _ in range(4):
            a.append(t(gs))
            b.append(t(gb))
        a.sort()
        b.sort()
        print(f"first {k:2d} launches (to {p1.steps[k - 1].what}): {'4 bs8 branches' if s4 else 'bs32 one pass'} "
              f"{a[1]:8.1f} us, "
              f"two bs16 branches {b[1]:8.1f} us  ({100 * (a[1] / b[1] - 1):+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
