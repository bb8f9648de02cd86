"""Sub-batch graphs on CU-partitioned streams: the two (or more) sub-batch plans of a split DetectSession as one graph
each, replayed on streams created with hipExtStreamCreateWithCUMask so the branches run on disjoint sets of CUs and
do not contend for the same CUs (their launches are latency-bound and few-workgroup), against the session's own
one-graph-two-branches launch.  Alternating rounds, same session buffers.

    python scripts/cu_mask_probe.py [--model n] [--batch 32] [--streams 2] [--split even|half]
"""
import argparse
import ctypes as C
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))

from bench import CFGS  # noqa: E402
from ydbl import YOLO  # noqa: E402
from ydbl.runtime import GraphRunner  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402


def masked_stream(hip, dev, cus):
    """A HIP stream limited to the CU indices in `cus` (hipExtStreamCreateWithCUMask), as a torch ExternalStream."""
    words = [0] * 8
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    arr = (C.c_uint32 * 8)(*words)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(8), arr)
    assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
    return torch.cuda.ExternalStream(s.value, device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg, wfile = CFGS[a.model][:2]
    model = YOLO(cfg, nc=3)
    load_trained(model.model, ROOT / "tests" / "golden" / wfile)
    sess = model.session(a.batch, 640, 640, half=True, conf=0.25, iou=0.7, max_det=300, device=dev, streams=a.streams)
    sess.load(blob_images(a.batch, 640, seed=1234).to(dev))
    for _ in range(5):
        sess.launch()
    torch.cuda.synchronize(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    hip = C.CDLL("libamdhip64.so")
    runners = [GraphRunner(c.plan) for c in sess.children]
    k = len(runners)
    layouts = {
        "plain": [torch.cuda.Stream(dev) for _ in runners],
        "interleaved": [masked_stream(hip, dev, [c for c in range(ncu) if c % k == i]) for i in range(k)],
        "blocks": [masked_stream(hip, dev, [c for c in range(ncu) if c * k // ncu == i]) for i in range(k)],
    }

    def two_graphs(streams):
        cur = torch.cuda.current_stream(dev)
        for r, st in zip(runners, streams):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                r.replay()
        for st in streams:
            cur.wait_stream(st)

    def t(fn, n=50):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n * 1e3

    print(f"{a.model} bs{a.batch} {k} sub-batch graphs, {ncu} CUs", flush=True)
    for r in range(a.rounds):
        row = {"session (one graph, branches)": t(sess.launch)}
        for name, st in layouts.items():
            row[f"{k} graphs, {name} streams"] = t(lambda st=st: two_graphs(st))
        print(f"round {r}: " + "  ".join(f"{n} {ms:.3f} ms ({a.batch / ms * 1e3:.0f} img/s)" for n, ms in row.items()),
              flush=True)


if __name__ == "__main__":
    main()
