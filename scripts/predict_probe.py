"""Host cost of YOLO.predict(x) on an HBM-resident bs32 batch (DBL-n 640 fp16): per-call host time without waiting
for the GPU, against the step time of the same calls back to back (GPU-bound when host < step).

    python scripts/predict_probe.py
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


def main():
    cfg, fx = CFGS["n"]
    torch.manual_seed(0)
    m = YOLO(cfg, nc=3)
    load_trained(m.model, ROOT / "tests" / "golden" / fx)
    x = blob_images(32, 640, seed=1234).cuda()
    for _ in range(10):
        m.predict(x, half=True)
    torch.cuda.synchronize()
    n = 50
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        m.predict(x, half=True)
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    host.sort()
    print(f"predict bs32: step {el / n * 1e3:.3f} ms, host per call median {host[n // 2] * 1e3:.3f} ms "
          f"(min {host[0] * 1e3:.3f}, max {host[-1] * 1e3:.3f})")
    s = list(m._sessions.values())[-1]
    t0 = time.perf_counter()
    for _ in range(n):
        s.launch()
    torch.cuda.synchronize()
    print(f"session replay alone: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per step")


if __name__ == "__main__":
    main()
