"""Per-launch in-graph profile of one compiled inference plan (forward + decode + NMS).

    python scripts/layer_profile.py [--model n] [--batch 32] [--imgsz 640] [--fp32] [--top 40]

Prints one line per launch: index, kernel, label, output shape, us, algorithmic GB/s.
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from bench import CFGS, conv_traffic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    from ydbl import YOLO
    from ydbl.utils.synthetic import blob_images, load_trained

    cfg, fx = CFGS[a.model]
    torch.manual_seed(0)
    m = YOLO(cfg, nc=3)
    load_trained(m.model, ROOT / "tests" / "golden" / fx)
    s = m.session(a.batch, a.imgsz, a.imgsz, half=not a.fp32, conf=0.25, iou=0.7, use_graph=False)
    s.load(blob_images(a.batch, a.imgsz, seed=1234).cuda())
    el = 4 if a.fp32 else 2
    best = s.plan.run_graph_timed()
    rows = []
    for i, (st, (what, ms)) in enumerate(zip(s.plan.steps, best)):
        kind = st.fn.__name__.replace("ydbl_", "")
        shape, gbs = "", ""
        d0 = st.args[0] if st.args else None
        if hasattr(d0, "x") and hasattr(d0, "y") and hasattr(d0.x, "c") and kind not in ("conv2d_nhwc", "dwconv2d_nhwc"):
            shape = f"{d0.x.c}x{d0.x.h}x{d0.x.w}->{d0.y.c}x{d0.y.h}x{d0.y.w}"
        if kind in ("conv2d_nhwc", "dwconv2d_nhwc"):
            d = st.args[0]
            shape = f"{d.x.c}x{d.x.h}x{d.x.w}->{d.y.c}x{d.y.h}x{d.y.w} k{d.kh} s{d.stride} d{d.dil}"
            if kind == "conv2d_nhwc":
                b, f = conv_traffic(st, el)
                gbs = f"{b / (ms * 1e-3) / 1e9:7.0f} GB/s {f / (ms * 1e-3) / 1e12:6.1f} TF"
            else:
                b = (d.x.n * d.x.h * d.x.w * d.x.c + d.y.n * d.y.h * d.y.w * d.y.c) * el
                gbs = f"{b / (ms * 1e-3) / 1e9:7.0f} GB/s"
        rows.append((i, kind, what, shape, ms * 1e3, gbs))
    total = sum(r[4] for r in rows)
    print(f"total {total:.1f} us over {len(rows)} launches  ({a.batch * 1e6 / total:.0f} img/s in-graph sum)")
    by = {}
    for r in rows:
        by[r[1]] = by.get(r[1], 0) + r[4]
    for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"  {k:24s} {v:9.1f} us {100 * v / total:5.1f}%")
    print("--- all launches in order")
    for r in rows:
        print(f"{r[0]:4d} {r[1]:18s} {r[2][:28]:28s} {r[3]:40s} {r[4]:8.1f} us  {r[5]}")


if __name__ == "__main__":
    main()
