"""Phase offset between the two sub-batch branches of the bench's one-graph layout (DBL-n bs32 fp16 640, streams=2):
branch 1 starts only after branch 0 has run its first K launches, so that the two branches' compute-bound
(stem pair, Bottlenecks) and memory- / latency-bound layers overlap instead of running in lockstep.  Each K is
captured as its own graph (the same plans and buffers as runtime.BranchGraphRunner) and replayed alternately
with the others; prints ms per step per K, several rounds.

    python scripts/branch_offset_probe.py [K ...]
"""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))

from ydbl import YOLO  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402


def run_steps(plan, steps, stream):
    import ctypes as C

    from ydbl import _lib

    s = C.c_void_p(stream)
    for st in steps:
        rc = st.fn(*st.args, s)
        if rc:
            _lib.check(rc, st.what)


def offset_graph(plans, k, dev):
    """plans[0]'s first k launches, then plans[1] on a side stream beside plans[0]'s rest (k = 0: the session's own
    fork at the start)."""
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream(dev)
        run_steps(plans[0], plans[0].steps[:k], cap.cuda_stream)
        side.wait_stream(cap)
        with torch.cuda.stream(side):
            run_steps(plans[1], plans[1].steps, side.cuda_stream)
        run_steps(plans[0], plans[0].steps[k:], cap.cuda_stream)
        cap.wait_stream(side)
    torch.cuda.synchronize(dev)
    return g


def main():
    ks = [int(a) for a in sys.argv[1:]] or [0, 1, 2, 3, 4, 6, 9]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = YOLO("yolov13n_DBL.yaml", nc=3)
    load_trained(model.model, ROOT / "tests" / "golden" / "trained_yolov13n_DBL_nc3.npz")
    sess = model.session(32, 640, 640, half=True, conf=0.25, iou=0.7, max_det=300, device=dev, streams=2)
    sess.load(blob_images(32, 640, seed=1234).to(dev))
    for _ in range(3):
        sess.launch()
    torch.cuda.synchronize(dev)
    plans = sess.plans
    print("branch 0 launches:", ", ".join(f"{i}:{st.what}" for i, st in enumerate(plans[0].steps[:12])), flush=True)
    graphs = {k: offset_graph(plans, k, dev) for k in ks}

    def t(g, n=40):
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n * 1e3

    res = {k: [] for k in ks}
    for r in range(4):
        for k in ks:
            res[k].append(t(graphs[k]))
    for k in ks:
        v = sorted(res[k])
        print(f"offset K={k:2d}: ms/step median {v[len(v) // 2]:.4f} best {v[0]:.4f}  "
              f"({32 / v[len(v) // 2] * 1e3:.0f} img/s)", flush=True)


if __name__ == "__main__":
    main()
