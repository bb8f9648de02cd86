"""Timing of ydbl_batch_max (predict()'s LoadTensor maximum) on the bench batch, 32x3x640x640 fp32, by variant
against torch.amax.  Warm = the batch still in the 256 MiB Infinity Cache (back-to-back calls); cold = a 512 MB
write between calls evicts it, as the network's activations do between two predict() calls.  --variants also
times the read orders of scripts/bmax_variants.hip (built with hipcc into abtmp/).

    python scripts/bmax_bench.py [--variants]
"""
import ctypes
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


def timed_cold(fn, flush, reps=40):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    ts = []
    for _ in range(reps):
        flush.fill_(1.0)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    x = torch.rand(32, 3, 640, 640, device="cuda")
    work = _lib.batch_max_work("cuda")
    amax, scale = torch.empty(1, device="cuda"), torch.empty(1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: _lib.lib.ydbl_batch_max(x.data_ptr(), x.numel(), work.data_ptr(), amax.data_ptr(), scale.data_ptr(), st)
    us = timed(f)
    print(f"ydbl_batch_max: {us:7.2f} us  ({x.numel() * 4 / us / 1e6:.2f} TB/s)", flush=True)
    print(f"torch.amax: {timed(lambda: torch.amax(x)):7.2f} us", flush=True)
    flush = torch.empty(128 * 1024 * 1024, device="cuda")
    tb = lambda us: x.numel() * 4 / us / 1e6
    us = timed_cold(f, flush)
    print(f"cold ydbl_batch_max: {us:7.2f} us  ({tb(us):.2f} TB/s)", flush=True)
    us = timed_cold(lambda: torch.amax(x), flush)
    print(f"cold torch.amax: {us:7.2f} us  ({tb(us):.2f} TB/s)", flush=True)
    if "--variants" not in sys.argv:
        return
    so = ctypes.CDLL(str(ROOT / "abtmp" / "libbmax_variants.so"))
    so.bmax_variant.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    part = torch.empty(1 << 20, device="cuda")
    ref = torch.amax(x).item()
    names = {0: "contiguous", 1: "staggered", 2: "interleaved", 3: "contiguous-nt", 4: "nt+atomics", 5: "nt+keys"}
    vwork = torch.zeros(260 * 64, dtype=torch.int32, device="cuda")
    vwork.view(-1, 64)[0::2] = -2 ** 31
    # (mode, rounds, blocks, skew | groups)
    cases = [(0, 16, 1200, 0), (0, 8, 4800, 0), (2, 8, 4096, 0), (3, 16, 1200, 0), (3, 8, 2400, 0), (3, 32, 600, 0),
             (3, 16, 600, 0), (3, 8, 1200, 0), (3, 16, 2400, 0), (3, 8, 4800, 0), (3, 32, 1200, 0),
             (4, 16, 1200, 8), (4, 16, 1200, 32), (4, 16, 600, 8), (4, 32, 600, 16), (4, 8, 2400, 32)]
    if "--atomics" in sys.argv:  # the merge's group count at the larger grids
        cases = [(3, 8, 4800, 0), (3, 8, 9600, 0), (3, 4, 9600, 0), (4, 8, 4800, 8), (4, 8, 4800, 32),
                 (4, 8, 4800, 64), (4, 8, 2400, 32), (4, 16, 2400, 32), (4, 16, 1200, 32), (4, 8, 9600, 64),
                 (5, 16, 1200, 8), (5, 16, 1200, 32), (5, 8, 4800, 32), (5, 4, 9600, 64), (5, 4, 9600, 8)]
    for mode, rounds, blocks, skew in cases:
        g = lambda: so.bmax_variant(mode, rounds, x.data_ptr(), x.numel(), blocks, skew, part.data_ptr(),
                                    vwork.data_ptr(), st)
        us = timed_cold(g, flush)
        part.fill_(-1.0)
        g()
        if mode == 5:  # the keys hold order keys of non-negative maxima: the float bits themselves
            keys = vwork[:skew * 64:64].clone()
            vwork[:skew * 64:64] = -2 ** 31
            g()
            got = vwork[:skew * 64:64].view(torch.float32).max()
            vwork.view(-1, 64)[0::2] = -2 ** 31
            vwork.view(-1, 64)[1::2] = 0
            ok = got.item() == ref
        else:
            ok = (part[0] if mode == 4 else torch.amax(part)).item() == ref
        print(f"cold {names[mode]:13s} R={rounds:2d} blocks={blocks:5d} skew={skew:4d}: {us:7.2f} us "
              f"({tb(us):.2f} TB/s) {'ok' if ok else 'WRONG'}", flush=True)


if __name__ == "__main__":
    main()
