"""Two sub-batch plans as two graphs on two streams (the bench's DetectSession(streams=2)) vs ONE hipGraph holding
both plans as independent branches (captured with a fork / join across a side stream), DBL-n bs32 fp16 640.
Prints ms per step for each, alternating, on the same session buffers."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))

from ydbl import YOLO  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = YOLO("yolov13n_DBL.yaml", nc=3)
    load_trained(model.model, ROOT / "tests" / "golden" / "trained_yolov13n_DBL_nc3.npz")
    sess = model.session(32, 640, 640, half=True, conf=0.25, iou=0.7, max_det=300, device=dev, streams=2)
    sess.load(blob_images(32, 640, seed=1234).to(dev))
    for _ in range(5):
        sess.launch()  # the session's own path: one graph with the two plans as branches (BranchGraphRunner)
    torch.cuda.synchronize(dev)
    # the round-3/4 path: one graph per sub-batch plan, each replayed on its own stream, joined per step
    from ydbl.runtime import GraphRunner

    runners = [GraphRunner(c.plan) for c in sess.children]
    streams = [torch.cuda.Stream(dev) for _ in runners]

    def two_graphs():
        cur = torch.cuda.current_stream(dev)
        for r, st in zip(runners, streams):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                r.replay()
        for st in streams:
            cur.wait_stream(st)

    def t(fn, n=50):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n * 1e3

    for r in range(3):
        a = t(two_graphs)
        b = t(sess.launch)
        print(f"round {r}: two graphs on two streams {a:.3f} ms/step ({32 / a * 1e3:.0f} img/s), "
              f"one graph with two branches {b:.3f} ms/step ({32 / b * 1e3:.0f} img/s)", flush=True)


if __name__ == "__main__":
    main()
