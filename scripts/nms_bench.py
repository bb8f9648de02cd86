"""Time ydbl_pred_candidates + ydbl_nms on synthetic predictions with a controlled candidate count."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl.utils.ops import non_max_suppression  # noqa: E402


def pred(B, nc, A, frac, seed=0):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(B, 2, A, generator=g) * 600 + 20
    wh = torch.rand(B, 2, A, generator=g) * 80 + 4
    sc = torch.rand(B, nc, A, generator=g) * 0.2
    k = int(frac * A)
    sc[:, 0, :k] = 0.3 + 0.7 * torch.rand(B, k, generator=g)
    return torch.cat([xy, wh, sc], 1).cuda()


for n_cand in (0, 50, 400, 2000, 8000):
    p = pred(32, 3, 8400, n_cand / 8400)
    for _ in range(3):
        non_max_suppression(p, 0.25, 0.7)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        r = non_max_suppression(p, 0.25, 0.7)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"cands/img {n_cand:5d}: {ev[0].elapsed_time(ev[1]) / 10 * 1e3:8.1f} us per call (cand+nms+readback), kept {len(r[0])}")
