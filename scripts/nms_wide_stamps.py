"""Round 6: phase timing of the NMS sweep kernel from the diagnostic build (scripts/build_stamps.sh detect):
per image workgroup on the pair-matrix path: prologue, then per-chunk phase sums a row staging / b block sweep /
c kept rows into later chunks."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["YDBL_LIB"] = str(ROOT / "scripts" / "bin" / "libydbl_detect_stamps.so")  # copy of build_dbg/ (gpurun-ignored)
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT / "scripts"))
sys.argv = [sys.argv[0], "-"]  # nms_wide_bench: definitions only
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ydbl import _lib  # noqa: E402
from ydbl._lib import NmsDesc, PredCandDesc  # noqa: E402

src = (ROOT / "scripts" / "nms_wide_bench.py").read_text().split("if len(sys.argv) > 1:")[0]
ns = {"__name__": "nms_wide_bench", "__file__": str(ROOT / "scripts" / "nms_wide_bench.py")}
exec(compile(src, "nms_wide_bench.py", "exec"), ns)
pred, cases = ns["pred"], ns["cases"]
for label, counts, nc, A, size in cases:
    B = len(counts)
    p = pred(B, nc, A, counts, size).float().contiguous()
    cb = torch.empty((B, A, 4), device="cuda"); cs = torch.empty((B, A), device="cuda")
    cc = torch.empty((B, A), dtype=torch.int32, device="cuda"); ci = torch.empty((B, A), dtype=torch.int32, device="cuda")
    cn = torch.zeros((B,), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib.ydbl_pred_candidates(PredCandDesc(p.data_ptr(), B, nc, A, 0.25, 0, None, 0, cb.data_ptr(),
                                                          cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(),
                                                          A), s))
    out = torch.zeros((B, 300, 6), device="cuda"); cnt = torch.zeros((B,), dtype=torch.int32, device="cuda")
    ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, A, 30000)), dtype=torch.uint8, device="cuda")
    nd = NmsDesc(cb.data_ptr(), cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(), B, A, 0.7, 300, 30000, 0,
                 7680.0, float(size), float(size), out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), 0, 0, 1)
    for _ in range(3):
        _lib.check(_lib.lib.ydbl_nms(nd, s))
    torch.cuda.synchronize()
    buf = np.zeros(16 * 4096, dtype=np.uint64)
    assert _lib.lib.ydbl_nms_debug_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), len(buf)) == 0
    st = buf.reshape(-1, 16)[:B].astype(np.int64)
    tot = (st[:, 3] - st[:, 0]) / 100.0
    i = int(np.argmax(tot))
    print(f"{label}: slowest wg {i} (m={st[i, 6]}, chunks {st[i, 5]}): total {tot[i]:.1f} us, prologue "
          f"{(st[i, 1] - st[i, 0]) / 100:.1f}; a/b/c {st[i, 7] / 100:.1f}/{st[i, 8] / 100:.1f}/{st[i, 9] / 100:.1f} us; "
          f"output {(st[i, 3] - st[i, 2]) / 100:.1f} us", flush=True)
