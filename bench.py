"""Benchmark: YOLO-DBL inference (forward + decode + NMS) images/sec on MI355X.

Default workload = BASELINE.json configs[1]: YOLO-DBL-n, 640x640, bs=32 per GPU,
fp16, predict settings (conf 0.25, iou 0.7, max_det 300), synthetic blob images
already resident in HBM, trained-like synthetic weights (tests/golden fixture).
A step = one hipGraph replay of forward + decode + NMS over the batch, plus (N>1)
one RCCL all-gather of the fixed-shape [B,300,6] box buffers.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model n|s|l] [--batch B] [--imgsz S] [--fp32]

N>1: launched by torch.distributed.run, one process per GPU; weak scaling
(B images per GPU), max-over-ranks time, value = all images / time.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_PEAK_TFLOPS = {"fp16": 2500.0, "fp32": 157.3, "fp8": 5000.0}
CFGS = {"n": ("yolov13n_DBL.yaml", "trained_yolov13n_DBL_nc3.npz"),
        "s": ("yolov13s_DBL.yaml", "trained_yolov13s_DBL_nc3.npz"),
        "l": ("yolov13l_DBL2.yaml", "trained_yolov13l_DBL2_nc3.npz")}


def conv_traffic(step, elsize):
    """Algorithmic bytes / FLOPs of one ydbl_conv2d_nhwc launch from its descriptor."""
    d = step.args[0]
    x, y = d.x, d.y
    cin = x.c
    k = d.kh * d.kw
    wsize = 1 if d.dq else elsize  # e4m3 weights in fp8 mode
    byts = (x.n * x.h * x.w * cin + y.n * y.h * y.w * y.c) * elsize + y.c * k * cin * wsize
    if d.res_mode:
        byts += y.n * y.h * y.w * y.c * elsize
    if d.y2.ptr:  # fused FullPAD: second output written + its other input read
        byts += 2 * y.n * y.h * y.w * y.c * elsize
    flops = 2.0 * y.n * y.h * y.w * y.c * k * cin
    return byts, flops


def roofline(session, dtype_name, reps=3):
    """Per-launch HIP-event timing of one eager forward; dominant kernel = the dense conv."""
    plan = session.plan
    elsize = 4 if dtype_name == "fp32" else 2  # activation bytes (fp8 mode keeps fp16 activations)
    best = None
    for _ in range(reps):
        t = plan.run_timed()
        if best is None:
            best = t
        else:
            best = [(w, min(a, b)) for (w, a), (_, b) in zip(best, t)]
    conv_ms = conv_bytes = conv_flops = 0.0
    by_kind = {}
    n_conv = 0
    for st, (what, ms) in zip(plan.steps, best):
        kind = st.fn.__name__
        by_kind[kind] = by_kind.get(kind, 0.0) + ms
        if kind == "ydbl_conv2d_nhwc":
            b, f = conv_traffic(st, elsize)
            conv_ms += ms
            conv_bytes += b
            conv_flops += f
            n_conv += 1
    total_ms = sum(ms for _, ms in best)
    ach_gbs = conv_bytes / (conv_ms * 1e-3) / 1e9
    ach_tf = conv_flops / (conv_ms * 1e-3) / 1e12
    ai = conv_flops / conv_bytes
    ridge = MFMA_PEAK_TFLOPS[dtype_name] * 1e12 / (HBM_PEAK_GBS * 1e9)
    bound = "hbm" if ai < ridge else "mfma"
    if bound == "hbm":
        rf = {"bound": "hbm", "achieved": round(ach_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(ach_gbs / HBM_PEAK_GBS, 4)}
    else:
        pk = MFMA_PEAK_TFLOPS[dtype_name]
        rf = {"bound": "mfma", "achieved": round(ach_tf, 2), "peak": pk, "unit": "TFLOP/s", "frac": round(ach_tf / pk, 4)}
    rf.update({"kernel": "ydbl_conv2d_nhwc", "launches_per_step": n_conv,
               "avg_launch_us": round(conv_ms * 1e3 / max(n_conv, 1), 2),
               "alg_bytes_per_launch": int(conv_bytes / max(n_conv, 1)),
               "alg_flops_per_step": conv_flops, "arith_intensity": round(ai, 1), "tflops": round(ach_tf, 2),
               "eager_step_ms": round(total_ms, 3),
               "ms_by_kernel": {k: round(v, 3) for k, v in sorted(by_kind.items(), key=lambda kv: -kv[1])}})
    rf["traffic"] = pmc_traffic()
    return rf


def pmc_traffic():
    """HBM bytes per conv launch from the committed rocprofv3 PMC summary (gfx950-corrected), if present."""
    p = ROOT / "profiles" / "pmc_conv_summary.json"
    if p.exists():
        try:
            return json.loads(p.read_text()).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def cpu_baseline(model_key, imgsz, budget_s=15.0):
    """Oracle (CPU restatement of the reference path, fp32) on a bounded sample: forward + NMS per image."""
    sys.path.insert(0, str(ROOT))
    from oracle.model import build_model
    from oracle.ops import non_max_suppression
    from ydbl.utils.synthetic import blob_images, load_trained

    cfg, fx = CFGS[model_key]
    torch.manual_seed(0)
    m = build_model(cfg, nc=3)
    load_trained(m, ROOT / "tests" / "golden" / fx)
    m.fuse()
    x = blob_images(1, imgsz, seed=1234)
    with torch.inference_mode():
        y, _ = m(x)  # warm-up
        non_max_suppression(y, 0.25, 0.7)
        n, t0 = 0, time.perf_counter()
        while True:
            y, _ = m(x)
            non_max_suppression(y, 0.25, 0.7)
            n += 1
            el = time.perf_counter() - t0
            if el > budget_s or n >= 200:
                break
    return {"value": round(n / el, 3), "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} images of {imgsz}x{imgsz}, bs=1, fp32 oracle forward+NMS ({el:.1f}s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="n", choices=list(CFGS))
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="e4m3 dense-conv operands (BASELINE config 5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from ydbl import YOLO
    from ydbl.utils.synthetic import blob_images, load_trained

    cfg, fx = CFGS[args.model]
    half = not args.fp32
    dtype_name = "fp8" if args.fp8 else ("fp16" if half else "fp32")
    torch.manual_seed(0)
    model = YOLO(cfg, nc=3)
    load_trained(model.model, ROOT / "tests" / "golden" / fx)
    B, S = args.batch, args.imgsz
    sess = model.session(B, S, S, half=half, conf=0.25, iou=0.7, max_det=300, device=dev, fp8=args.fp8)
    if args.fp8:  # activation scales from a separate synthetic calibration batch
        sess.calibrate_fp8(blob_images(B, S, seed=4321 + rank).to(dev))
    # synthetic images, different per rank, resident in the session's input buffer (HBM)
    sess.load(blob_images(B, S, seed=1234 + rank).to(dev))
    from ydbl.parallel import gather_detections

    def step():
        det, cnt = sess()  # this rank's B images: forward + decode + NMS (one hipGraph replay)
        if world > 1:  # the path's only exchange: one all-gather of the fixed-shape box buffers
            gather_detections(det, cnt, B * world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    images = B * world * args.steps
    value = images / el
    dets_per_img = float(sess.count.float().mean().item())
    cands_per_img = float(sess.cand_count.float().mean().item())
    cands_max = int(sess.cand_count.max().item())

    rf = None
    if rank == 0 and not args.no_roofline:
        rf = roofline(sess, dtype_name)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.model, S)
    if rank == 0:
        out = {
            "metric": "images/sec @640×640 bs=32 (1/2/4/8 GPU) + mAP@0.5 vs CPU ref",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype_name,
            "data": "synthetic (blob images, trained-like synthetic weights tests/golden)",
            "config": {"workload": f"YOLO-DBL-{args.model} {S}x{S} bs={B}/GPU {dtype_name} forward+decode+NMS "
                                   f"(conf .25, iou .7, max_det 300)" + (", RCCL all-gather of boxes" if world > 1 else ""),
                       "model": Path(cfg).stem, "global_batch": B * world, "imgsz": S, "nc": 3,
                       "parallelism": f"dp{world}"},
            "dets_per_image": round(dets_per_img, 2),
            "candidates_per_image": round(cands_per_img, 1),
            "candidates_max": cands_max,
            "roofline": rf,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
