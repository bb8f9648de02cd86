"""DSBottleneck(64) at DBL-n's 40x40 bs32: fused ydbl_dsbottleneck_nhwc vs the two DSConv launches."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-dbl_amd")]
import torch  # noqa: E402

from ydbl.nn import modules as M  # noqa: E402
from ydbl.runtime import Plan  # noqa: E402
sys.path.insert(0, str(ROOT / "scripts"))
from conv_bench_util import bench  # noqa: E402

modes = sys.argv[1:] or ["fused", "two"]
for mode in modes:
    for (B, H) in ((32, 40), (64, 40)):
        plan = Plan(torch.device("cuda"), torch.float16)
        x = plan.alloc(B, H, H, 64)
        x.torch().copy_(torch.randn(B, H, H, 64, dtype=torch.float16))
        m = M.DSBottleneck(64, 64, shortcut=True, e=1.0, k1=3, k2=7).eval()
        if mode == "fused":
            os.environ["YDBL_DSBNECK"] = "1"
        m.emit(plan, x)
        os.environ.pop("YDBL_DSBNECK", None)
        t = bench(plan)
        print(f"DSBottleneck(64) {mode:5s} B{B} @{H}: {t:7.1f} us ({len(plan.steps)} launches)", flush=True)
