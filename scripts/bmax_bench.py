"""Timing of ydbl_batch_max (predict()'s LoadTensor maximum) on the bench batch, 32x3x640x640 fp32, by variant
against torch.amax.

    python scripts/bmax_bench.py
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))

import torch  # noqa: E402

from ydbl import _lib  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


def main():
    x = torch.rand(32, 3, 640, 640, device="cuda")
    work = _lib.batch_max_work("cuda")
    amax, scale = torch.empty(1, device="cuda"), torch.empty(1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: _lib.lib.ydbl_batch_max(x.data_ptr(), x.numel(), work.data_ptr(), amax.data_ptr(), scale.data_ptr(), st)
    us = timed(f)
    print(f"ydbl_batch_max: {us:7.2f} us  ({x.numel() * 4 / us / 1e6:.2f} TB/s)", flush=True)
    print(f"torch.amax: {timed(lambda: torch.amax(x)):7.2f} us", flush=True)


if __name__ == "__main__":
    main()
