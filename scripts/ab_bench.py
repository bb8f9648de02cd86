"""A/B of YDBL_* routing knobs on the bench workload in ONE process (same box, interleaved rounds), so box-to-box
spread does not enter the comparison.  Each variant is a separate session (the session key holds the knobs).

    python scripts/ab_bench.py "A:" "B:YDBL_CV3_FUSE=1;YDBL_NO_MERGE=1" [--model n] [--batch 32] [--streams 2] [--rounds 5]
    python scripts/ab_bench.py "S2:" "S3:STREAMS=3" "S4:STREAMS=4"        (sub-batch graphs per variant)
A variant listed twice under two names ("A:" ... "A2:") is two sessions with the same routing: their spread is the
session-to-session bias (buffer placement), about 0.5 % on DBL-n bs32 (profiles/r06/r06_defaults_ab.txt).
"""
import argparse
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from bench import CFGS  # noqa: E402


def parse(spec):
    name, _, rest = spec.partition(":")
    env = dict(kv.split("=", 1) for kv in rest.split(";") if kv)  # K=V;K2=V2 (values may hold commas)
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--model", default="n")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    from ydbl import YOLO
    from ydbl.utils.synthetic import blob_images, load_trained

    cfg, fx = CFGS[a.model]
    torch.manual_seed(0)
    model = YOLO(cfg, nc=3)
    load_trained(model.model, ROOT / "tests" / "golden" / fx)
    x = blob_images(a.batch, a.imgsz, seed=1234).cuda()
    base = {k: v for k, v in os.environ.items() if k.startswith("YDBL_")}
    sess = {}
    for spec in a.variants:
        name, env = parse(spec)
        streams = int(env.pop("STREAMS", a.streams))  # "S3:STREAMS=3": sub-batch graphs of this variant
        for k in [k for k in os.environ if k.startswith("YDBL_")]:
            del os.environ[k]
        os.environ.update(base)
        os.environ.update(env)
        s = model.session(a.batch, a.imgsz, a.imgsz, half=True, conf=0.25, iou=0.7, streams=streams)
        s.load(x)
        for _ in range(5):
            s()
        torch.cuda.synchronize()
        n = sum(len(p.steps) for p in s.plans)
        sess[name] = (s, n)
    res = {k: [] for k in sess}
    for _ in range(a.rounds):
        for name, (s, _) in sess.items():
            for _ in range(3):  # untimed: the previous variant's buffers leave the caches first
                s()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                s()
            torch.cuda.synchronize()
            res[name].append(a.batch * a.steps / (time.perf_counter() - t0))
    for name, v in res.items():
        v = sorted(v)
        print(f"{name:12s} launches {sess[name][1]:4d}  img/s median {v[len(v) // 2]:9.1f}  best {v[-1]:9.1f}  "
              f"all {' '.join(f'{u:.0f}' for u in v)}", flush=True)


if __name__ == "__main__":
    main()
