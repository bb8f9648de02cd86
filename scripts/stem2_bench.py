"""Micro-benchmark: ydbl_conv_stem2 (layers 0+1 fused) vs ydbl_conv_stem + the unfused stride-2 conv."""
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


cases = [(32, 640, 640, 8), (32, 640, 640, 16), (64, 640, 640, 16)]
sel = [int(a) for a in sys.argv[1:]] or range(len(cases))
for ci in sel:
    B, H, W, c0 = cases[ci]
    plan = Plan(torch.device("cuda"), torch.float16)
    x = torch.rand(B, 3, H, W, device="cuda")
    w0, b0 = torch.randn(c0, 3, 3, 3) * 0.2, torch.randn(c0)
    w1, b1 = torch.randn(2 * c0, c0, 3, 3) * 0.1, torch.randn(2 * c0)
    host = torch.empty(int(_lib.lib.ydbl_conv_stem2_params_size(c0)), dtype=torch.uint8)
    _lib.check(_lib.lib.ydbl_conv_stem2_pack(w0.data_ptr(), b0.data_ptr(), w1.data_ptr(), b1.data_ptr(), c0,
                                             host.data_ptr()))
    params = host.cuda()
    y = plan.alloc(B, H // 2, W // 2, 2 * c0)
    d = _lib.Stem2Desc(x.data_ptr(), B, 3, H, W, 1.0, c0, params.data_ptr(), y.struct())
    s = torch.cuda.current_stream().cuda_stream
    f2 = lambda: _lib.check(_lib.lib.ydbl_conv_stem2(d, s))
    # unfused: stem (3->c0 s1) + dense conv (c0 -> 2c0 s2)
    mid = plan.alloc(B, H, W, c0)
    wd, bd = w0.cuda(), b0.cuda()
    ms = mid.struct()
    f_stem = lambda: _lib.lib.ydbl_conv_stem(x.data_ptr(), B, 3, H, W, 1.0, wd.data_ptr(), bd.data_ptr(), 3, 1, 1, ms, None, s)
    p2 = Plan(torch.device("cuda"), torch.float16)
    emit_dense(p2, mid, y, w1, b1, 2, 1, 1, _lib.ACT_SILU)
    f_conv = lambda: p2.run()
    mb = (B * 3 * H * W * 4 + B * (H // 2) * (W // 2) * 2 * c0 * 2) / 1e6
    t2, ts, tc = bench(f2), bench(f_stem), bench(f_conv)
    print(f"B{B} {H}x{W} c0={c0}: stem2 {t2:7.1f} us ({mb / t2:5.2f} TB/s of in+out)   "
          f"unfused stem {ts:6.1f} + conv {tc:6.1f} = {ts + tc:6.1f} us", flush=True)
