"""Micro-benchmark of the fused DSConv launch on the DBL-n/s shapes (HIP-event timed, per tile config)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl.nn import modules as M  # noqa: E402
from ydbl.runtime import Plan  # noqa: E402

SHAPES = [  # (B, cin, cout, k, s, H, W)
    (32, 64, 64, 3, 1, 40, 40), (32, 64, 64, 7, 1, 40, 40), (32, 128, 128, 3, 2, 80, 80),
    (32, 128, 256, 3, 2, 40, 40), (32, 128, 128, 3, 1, 20, 20), (32, 128, 128, 7, 1, 20, 20),
    (32, 32, 32, 7, 1, 40, 40), (32, 128, 128, 7, 1, 40, 40),
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


for cfg in sys.argv[1:] or ["A"]:
    os.environ["YDBL_DS_TILE"] = cfg
    line = []
    for (B, ci, co, k, s, H, W) in SHAPES:
        plan = Plan(torch.device("cuda"), torch.float16)
        x = plan.alloc(B, H, W, ci)
        x.torch().copy_(torch.randn(B, H, W, ci, dtype=torch.float16))
        m = M.DSConv(ci, co, k, s).eval()
        m.emit(plan, x)
        line.append(f"{bench(plan):6.1f}")
    print(cfg, " ".join(line), flush=True)
