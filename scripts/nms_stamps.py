"""NMS phase timing from the diagnostic build (scripts/build_stamps.sh detect): per-workgroup
s_memrealtime stamps (100 MHz) at start / sorted / staged / swept, plus rounds and list length."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["YDBL_LIB"] = str(ROOT / "build_dbg" / "libydbl_stamps.so")
os.environ.setdefault("YDBL_NMS_GROUPS", "0")
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT / "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nms_bench as nb  # noqa: E402  (runs its own table first)
from ydbl import _lib  # noqa: E402

for label, counts, nc, spread in [("31 x 120 + 1 x 650", [120] * 31 + [650], 3, False),
                                  ("32 x 120", [120] * 32, 3, False), ("32 x 2000", [2000] * 32, 3, False)]:
    us, _ = nb.run(counts, nc=nc, spread=spread, reps=1)
    buf = np.zeros(16 * 4096, dtype=np.uint64)
    assert _lib.lib.ydbl_nms_debug_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), len(buf)) == 0
    st = buf.reshape(-1, 16)[:len(counts)].astype(np.int64)
    d = (st[:, 1:4] - st[:, 0:3]) / 100.0  # us
    tot = (st[:, 3] - st[:, 0]) / 100.0
    i = int(np.argmax(tot))
    print(f"{label}: launch {us:.1f} us; slowest wg {i}: sort {d[i,0]:.1f} stage {d[i,1]:.1f} sweep {d[i,2]:.1f} us "
          f"({st[i,5]} rounds, m={st[i,6]}); median wg total {np.median(tot):.1f} us; sweep phases a/b/c/d "
          f"{st[i,7]/100:.1f}/{st[i,8]/100:.1f}/{st[i,9]/100:.1f}/{st[i,10]/100:.1f} us", flush=True)
