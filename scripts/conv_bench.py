"""Micro-benchmark of ydbl_conv2d_nhwc on the DBL-n 3x3 / 1x1 shapes (HIP-event timed, fp16, bs 32).


"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl.nn import modules as M  # noqa: E402
from ydbl.runtime import Plan  # noqa: E402

SHAPES = [  # (cin, cout, k, s, H[, B])
    (384, 64, 3, 1, 40), (64, 128, 3, 1, 40), (256, 32, 3, 1, 80), (64, 64, 3, 2, 80), (192, 64, 3, 1, 40),
    (128, 128, 3, 2, 40), (64, 64, 3, 1, 80), (128, 64, 3, 1, 40), (64, 64, 3, 1, 40), (256, 64, 3, 1, 20),
    (64, 64, 3, 1, 20), (64, 32, 3, 1, 80),
    (64, 128, 1, 1, 80), (128, 64, 1, 1, 80), (64, 64, 1, 1, 80), (64, 64, 1, 1, 40), (128, 128, 1, 1, 40),
    (384, 128, 1, 1, 40), (512, 128, 1, 1, 40), (128, 64, 1, 1, 40), (384, 256, 1, 1, 20), (64, 3, 1, 1, 80),
    # DBL-s bs 64 / DBL-l 1280 bs 8 heavy hitters (indices 22..)
    (512, 64, 3, 1, 80, 64), (768, 128, 3, 1, 40, 64), (384, 128, 3, 1, 40, 64), (128, 128, 3, 1, 80, 64),
    (1024, 128, 3, 1, 160, 8), (128, 256, 3, 2, 320, 8), (64, 128, 3, 1, 320, 8), (1024, 256, 1, 1, 40, 64),
    (1280, 256, 1, 1, 160, 8), (2048, 512, 1, 1, 80, 8),
    (128, 192, 1, 1, 40), (320, 128, 1, 1, 40), (256, 128, 1, 1, 20), (128, 128, 1, 1, 20),  # 32..35
]


def bench(plan, reps=20):
    plan.run()
    torch.cuda.synchronize()
    torch.cuda._sleep(int(5e7))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        plan.run()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


sel = [int(a) for a in sys.argv[1:]]
for idx, shp in enumerate(SHAPES):
    if sel and idx not in sel:
        continue
    ci, co, k, s, H = shp[:5]
    B = shp[5] if len(shp) > 5 else int(os.environ.get("YDBL_BENCH_B", 32))
    plan = Plan(torch.device("cuda"), torch.float16)
    x = plan.alloc(B, H, H, ci)
    x.torch().copy_(torch.randn(B, H, H, ci, dtype=torch.float16))
    m = M.Conv(ci, co, k, s).eval()
    m.emit(plan, x)
    t = bench(plan)
    ho = H // s
    mb = (B * H * H * ci + B * ho * ho * co + co * ci * k * k) * 2 / 1e6
    tf = 2.0 * B * ho * ho * co * ci * k * k / 1e12
    print(f"B{B:3d} {ci:4d}->{co:4d} k{k} s{s} @{H:3d}: {t:7.1f} us  {mb / t:6.2f} TB/s  {tf / t * 1e6:7.1f} TF", flush=True)
