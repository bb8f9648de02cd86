"""DSConv launch times on the bench's bs16 sub-batch shapes for each tile configuration (YDBL_DS_TILE is read
once per process, so every configuration runs in its own child process).

    python scripts/ds_bench16.py [A 8 S]
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SHAPES = [  # (B, cin, cout, k, s, H, W)
    (16, 64, 64, 3, 1, 80, 80), (16, 64, 64, 3, 1, 40, 40), (16, 64, 64, 7, 1, 40, 40),
    (16, 128, 128, 3, 1, 20, 20), (16, 128, 128, 7, 1, 20, 20), (16, 256, 64, 3, 1, 20, 20),
    (16, 128, 64, 3, 1, 40, 40), (16, 64, 128, 3, 2, 80, 80),
]

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
    import torch

    from ydbl.nn import modules as M
    from ydbl.runtime import Plan

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

    line = []
    for (B, ci, co, k, s, H, W) in SHAPES:
        plan = Plan(torch.device("cuda"), torch.float16)
        x = plan.alloc(B, H, W, ci)
        x.torch().copy_(torch.randn(B, H, W, ci, dtype=torch.float16))
        m = M.DSConv(ci, co, k, s).eval()
        m.emit(plan, x)
        line.append(f"{bench(plan):6.1f}")
    print(os.environ.get("YDBL_DS_TILE", "A"), " ".join(line), flush=True)
else:
    print("shapes:", " ".join(f"{ci}->{co}k{k}s{s}@{H}" for (_, ci, co, k, s, H, W) in SHAPES), flush=True)
    for cfg in sys.argv[1:] or ["A"]:
        env = dict(os.environ, YDBL_DS_TILE=cfg)
        subprocess.run([sys.executable, __file__, "--child"], env=env, check=True)
