"""Micro-benchmark: ydbl_conv_stem vs the plain layout kernel on one image batch (HIP-event timed)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl import _lib  # noqa: E402
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


for (B, H, W, cout, dt) in [(32, 640, 640, 8, torch.float16), (32, 640, 640, 16, torch.float16),
                            (8, 1280, 1280, 32, torch.float16), (32, 640, 640, 8, torch.float32)]:
    plan = Plan(torch.device("cuda"), dt)
    x = torch.rand(B, 3, H, W, device="cuda")
    y = plan.alloc(B, H, W, cout)
    inp = plan.alloc(B, H, W, 8)
    wt = torch.randn(cout, 3, 3, 3, device="cuda")
    bs = torch.randn(cout, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    ys, ins = y.struct(), inp.struct()
    f1 = lambda: _lib.lib.ydbl_conv_stem(x.data_ptr(), B, 3, H, W, 1.0, wt.data_ptr(), bs.data_ptr(), 3, 1, 1, ys, s)
    f0 = lambda: _lib.lib.ydbl_conv_stem(x.data_ptr(), B, 3, H, W, 1.0, wt.data_ptr(), bs.data_ptr(), 3, 1, 0, ys, s)
    f2 = lambda: _lib.lib.ydbl_input_nchw_to_nhwc(x.data_ptr(), B, 3, H, W, 1.0, ins, s)
    es = 2 if dt == torch.float16 else 4
    mb = (B * 3 * H * W * 4 + B * H * W * cout * es) / 1e6
    t1, t0, t2 = bench(f1), bench(f0), bench(f2)
    print(f"B{B} {H}x{W} cout{cout} {dt}: stem silu {t1:7.1f} us ({mb / t1 * 1e-3:5.2f} TB/s)  stem no-act {t0:7.1f} us"
          f"  layout-only {t2:7.1f} us")
