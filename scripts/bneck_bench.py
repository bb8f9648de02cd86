"""Micro-benchmark: ydbl_bottleneck_nhwc (cv1 + cv2 + residual in one launch) vs the two dense-conv launches.

    python scripts/bneck_bench.py [case indices]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl import _lib  # noqa: E402
from ydbl.nn.modules import emit_dense  # noqa: E402
from ydbl.runtime import Plan  # noqa: E402


def bench(fn, reps=20):
    torch.cuda.synchronize()
    torch.cuda._sleep(int(5e7))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


# (batch, h, w, c): DBL-n backbone L2 / L4 / L6, DBL-s L2 / L4, DBL-l(1280) L2
cases = [(32, 320, 320, 16), (32, 160, 160, 32), (32, 80, 80, 64), (64, 320, 320, 32), (64, 160, 160, 64),
         (8, 640, 640, 64)]
sel = [int(a) for a in sys.argv[1:]] or range(len(cases))
for ci in sel:
    B, H, W, c = cases[ci]
    cm = c // 2
    plan = Plan(torch.device("cuda"), torch.float16)
    x = plan.alloc(B, H, W, c)
    x.torch().copy_(torch.randn(B, H, W, c, device="cuda").half())
    y = plan.alloc(B, H, W, c)
    w1, b1 = torch.randn(cm, c, 3, 3) / (9 * c) ** 0.5, torch.randn(cm) * 0.5
    w2, b2 = torch.randn(c, cm, 3, 3) / (9 * cm) ** 0.5, torch.randn(c) * 0.5
    host = torch.empty(int(_lib.lib.ydbl_bottleneck_params_size(c)), dtype=torch.uint8)
    _lib.check(_lib.lib.ydbl_bottleneck_pack(w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), c,
                                             host.data_ptr()))
    params = host.cuda()
    s = torch.cuda.current_stream().cuda_stream
    ds = {th: _lib.BottleneckDesc(x.struct(), y.struct(), c, 1, th, params.data_ptr()) for th in (8, 16)}
    mid = plan.alloc(B, H, W, cm)
    p1 = Plan(torch.device("cuda"), torch.float16)
    emit_dense(p1, x, mid, w1, b1, 1, 1, 1, _lib.ACT_SILU)
    p2 = Plan(torch.device("cuda"), torch.float16)
    emit_dense(p2, mid, y, w2, b2, 1, 1, 1, _lib.ACT_SILU, res=x, res_mode=_lib.RES_ADD)
    mb = 2 * B * H * W * c * 2 / 1e6
    gf = 2 * B * H * W * 2 * 9 * c * cm / 1e9
    tf = {th: bench(lambda: _lib.check(_lib.lib.ydbl_bottleneck_nhwc(ds[th], s))) for th in (8, 16)}
    t1, t2 = bench(lambda: p1.run()), bench(lambda: p2.run())
    best = min(tf.values())
    print(f"B{B} {H}x{W} c={c}: fused th8 {tf[8]:7.1f} us  th16 {tf[16]:7.1f} us  ({mb / best:5.2f} TB/s in+out, "
          f"{gf / best * 1e3:6.1f} TF)   unfused cv1 {t1:6.1f} + cv2 {t2:6.1f} = {t1 + t2:6.1f} us", flush=True)
