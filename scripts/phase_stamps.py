"""Phase timing from the diagnostic builds (scripts/build_stamps.sh bneck|stem2): per-workgroup s_memrealtime
stamps (100 MHz) when wave 0 starts / has staged the input window / has finished the first conv / has stored the
second, and the hardware ids (XCD, SE, CU).  Prints phase medians and how many workgroups each CU held at once.

    python scripts/bneck_stamps.py [--stem2] [c64@80 ...]   (kbench case substrings; default: the DBL-n backbone)
"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KIND = "stem2" if "--stem2" in sys.argv else "bneck"
os.environ["YDBL_LIB"] = str(ROOT / "build_dbg" / f"libydbl_{KIND}_stamps.so")
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT / "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kbench  # noqa: E402
from ydbl import _lib  # noqa: E402

sel = [a for a in sys.argv[1:] if a != "--stem2"] or (["stem2"] if KIND == "stem2" else
                                                      ["bneck c16@320", "bneck c32@160", "bneck c64@80", "box3 64@80"])
get, reset = getattr(_lib.lib, f"ydbl_{KIND}_debug_stamps"), getattr(_lib.lib, f"ydbl_{KIND}_debug_reset")
for name, build in kbench.CASES:
    if not any(s in name for s in sel):
        continue
    plan = build()
    for _ in range(2):
        plan.run()
    torch.cuda.synchronize()
    assert reset() == 0
    plan.run()
    torch.cuda.synchronize()
    n = 16384
    buf = np.zeros(8 * n, dtype=np.uint64)
    assert get(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), len(buf)) == 0
    st = buf.reshape(-1, 8).astype(np.int64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    t = (st[:, :4] - t0) / 100.0  # us
    hw, xcc = st[:, 4], st[:, 5]
    cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
    ph = np.diff(t, axis=1)
    print(f"{name}: {len(st)} workgroups, span {t[:, 3].max():.1f} us; start first->last {t[:, 0].max():.1f} us; "
          f"phase medians stage {np.median(ph[:, 0]):.2f} cv1 {np.median(ph[:, 1]):.2f} cv2 {np.median(ph[:, 2]):.2f} us "
          f"(p90 {np.percentile(ph[:, 0], 90):.2f} / {np.percentile(ph[:, 1], 90):.2f} / {np.percentile(ph[:, 2], 90):.2f}); "
          f"{len(np.unique(cu))} CUs", flush=True)
    # resident workgroups per CU: max over the launch (event sweep) and the time average over the span
    ids, inv = np.unique(cu, return_inverse=True)
    mx = 0
    for c in range(len(ids)):
        ev = sorted([(v, 1) for v in t[inv == c, 0]] + [(v, -1) for v in t[inv == c, 3]], key=lambda e: (e[0], e[1]))
        cur = 0
        for _, d in ev:
            cur += d
            mx = max(mx, cur)
    mean = (t[:, 3] - t[:, 0]).sum() / (len(ids) * t[:, 3].max())
    cnt = np.bincount(inv)
    print(f"   per-CU resident workgroups: max {mx}, mean over the span {mean:.2f}; workgroups per CU: min {cnt.min()} "
          f"max {cnt.max()}", flush=True)
    q = np.percentile(t[:, 0], [0, 25, 50, 75, 100])
    print("   start-time quartiles (us):", " ".join(f"{v:.1f}" for v in q), flush=True)
