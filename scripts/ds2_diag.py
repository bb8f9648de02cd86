"""Diagnose fused-vs-unfused DySample differences (fp16): variants with zero offset weights (offsets = bias only) or
zero bias, and the count/positions of differing outputs.

    python scripts/ds2_diag.py
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import torch  # noqa: E402

from test_gpu_ops import _plan, _tv_from_nchw, _run  # noqa: E402
from ydbl.nn import modules as M  # noqa: E402


def run(ds, x, fused, dtype):
    if fused:
        os.environ.pop("YDBL_DS2_OFF", None)
    else:
        os.environ["YDBL_DS2_OFF"] = "1"
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x)
    y = ds.emit(plan, xv)
    _run(plan)
    return y.nchw().float().cpu()


for name, wsd, bsd in [("weights 0", 0.0, 0.1), ("bias 0", 0.01, 0.0), ("both", 0.01, 0.1), ("big", 0.3, 3.0)]:
    for dtype in (torch.float16,):
        torch.manual_seed(1)
        c = 128
        ds = M.DySample(c)
        with torch.no_grad():
            ds.offset.weight.normal_(0, wsd) if wsd else ds.offset.weight.zero_()
            ds.offset.bias.normal_(0, bsd) if bsd else ds.offset.bias.zero_()
        x = torch.randn(2, c, 16, 16)
        a, b = run(ds, x, False, dtype), run(ds, x, True, dtype)
        d = (a != b)
        idx = d.nonzero()[:6].tolist()
        print(f"{name:10s} {dtype}: {int(d.sum())} of {d.numel()} differ, max {float((a - b).abs().max()):.3g}; first {idx}",
              flush=True)
        by_c = d.sum(dim=(0, 2, 3))
        print("   per channel-group:", [int(by_c[g * 32:(g + 1) * 32].sum()) for g in range(4)],
              " per (y%2,x%2):", [int(d[:, :, i::2, j::2].sum()) for i in range(2) for j in range(2)], flush=True)
