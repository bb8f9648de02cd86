"""Do two (or four) independent single-stream hipGraphs replayed on different HIP streams overlap?

The DBL-n bs32 step split into k sub-batches of 32/k images, one compiled session (own buffers, own
graph) per sub-batch, each replayed on its own stream; throughput vs the single bs32 graph.
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-dbl_amd")]
import torch  # noqa: E402

from bench import CFGS  # noqa: E402
from ydbl import YOLO  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402

model_key = sys.argv[1] if len(sys.argv) > 1 else "n"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
S = 640
cfg, fx = CFGS[model_key]
torch.manual_seed(0)
m = YOLO(cfg, nc=3)
load_trained(m.model, ROOT / "tests" / "golden" / fx)
x = blob_images(B, S, seed=1234).cuda()
for k in (1, 2, 4):
    b = B // k
    sess = [m.session(b, S, S, half=True, conf=0.25, iou=0.7) for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    for i, s in enumerate(sess):
        s.load(x[i * b:(i + 1) * b])
        s.launch()  # capture
    torch.cuda.synchronize()

    def step():
        cur = torch.cuda.current_stream()
        for s, st in zip(sess, streams):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                s.launch()
        for st in streams:
            cur.wait_stream(st)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    n = 40
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{model_key} bs{B} as {k} x bs{b} graphs on {k} streams: {el / n * 1e3:.3f} ms/step  {B * n / el:.0f} img/s",
          flush=True)
