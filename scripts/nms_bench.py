"""Time ydbl_nms alone (HIP events, 20 back-to-back launches) on synthetic candidates: bs 32 images
with a controlled candidate count per image (plus one heavy image, like the bench's max)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl import _lib  # noqa: E402
from ydbl._lib import NmsDesc, PredCandDesc  # noqa: E402


def pred(B, nc, A, counts, seed=0, spread=False):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(B, 2, A, generator=g) * 600 + 20
    wh = torch.rand(B, 2, A, generator=g) * 80 + 4
    sc = torch.rand(B, nc, A, generator=g) * 0.2
    for b, k in enumerate(counts):
        if spread:  # candidate i belongs to class i % nc
            for c in range(nc):
                idx = torch.arange(c, k, nc)
                sc[b, c, idx] = 0.3 + 0.7 * torch.rand(len(idx), generator=g)
        else:
            sc[b, 0, :k] = 0.3 + 0.7 * torch.rand(k, generator=g)
    return torch.cat([xy, wh, sc], 1).cuda()


def run(counts, nc=3, A=8400, reps=20, spread=False):
    B = len(counts)
    p = pred(B, nc, A, counts, spread=spread).float().contiguous()
    dev = p.device
    cap = A
    cb = torch.empty((B, cap, 4), device=dev); cs = torch.empty((B, cap), device=dev)
    cc = torch.empty((B, cap), dtype=torch.int32, device=dev); ci = torch.empty((B, cap), dtype=torch.int32, device=dev)
    cn = torch.zeros((B,), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    pd = PredCandDesc(p.data_ptr(), B, nc, A, 0.25, 0, None, 0, cb.data_ptr(), cs.data_ptr(), cc.data_ptr(),
                      ci.data_ptr(), cn.data_ptr(), cap)
    _lib.check(_lib.lib.ydbl_pred_candidates(pd, s))
    out = torch.zeros((B, 300, 6), device=dev); cnt = torch.zeros((B,), dtype=torch.int32, device=dev)
    ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, cap, 30000)), dtype=torch.uint8, device=dev)  # zero-filled once (include/ydbl.h)
    nd = NmsDesc(cb.data_ptr(), cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(), B, cap, 0.7, 300, 30000, 0,
                 7680.0, 640.0, 640.0, out.data_ptr(), cnt.data_ptr(), ws.data_ptr())
    _lib.check(_lib.lib.ydbl_nms(nd, s))
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e7))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        _lib.lib.ydbl_nms(nd, s)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3, cnt.tolist()


cases = [("32 x 0", [0] * 32, 3, False), ("32 x 120", [120] * 32, 3, False),
         ("31 x 120 + 1 x 650", [120] * 31 + [650], 3, False), ("32 x 650", [650] * 32, 3, False),
         ("32 x 2000", [2000] * 32, 3, False), ("31x120+1x650 nc3 spread", [120] * 31 + [650], 3, True),
         ("32 x 650 nc3 spread", [650] * 32, 3, True), ("32 x 2000 nc80 spread", [2000] * 32, 80, True)]
for label, counts, nc, spread in cases:
    us, kept = run(counts, nc=nc, spread=spread)
    print(f"{label:26s}: {us:8.1f} us per ydbl_nms launch   kept {kept[0]}..{kept[-1]}", flush=True)
