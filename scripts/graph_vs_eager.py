"""Is a hipGraph replay slower than the same launches enqueued eagerly behind a parked stream?
DBL-n bs32 fp16 one plan: (a) graph replay, (b) eager walk enqueued while the stream sleeps (no host
gaps between kernels), each timed with one event pair around the whole step."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-dbl_amd")]
import torch  # noqa: E402

from bench import CFGS  # noqa: E402
from ydbl import YOLO  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402

model_key = sys.argv[1] if len(sys.argv) > 1 else "n"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
cfg, fx = CFGS[model_key]
torch.manual_seed(0)
m = YOLO(cfg, nc=3)
load_trained(m.model, ROOT / "tests" / "golden" / fx)
s = m.session(B, 640, 640, half=True)
s.load(blob_images(B, 640, seed=1234).cuda())
s.launch()
torch.cuda.synchronize()
plan = s.plan
stream = torch.cuda.current_stream()


def timed(fn, n=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(2e8))
    a.record(stream)
    for _ in range(n):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for rep in range(2):
    g = timed(s.launch)
    e = timed(plan.run, n=3)
    print(f"graph replay {g:.3f} ms/step   eager (parked stream) {e:.3f} ms/step  ({len(plan.steps)} launches)",
          flush=True)
