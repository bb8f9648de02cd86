"""Benchmark: YOLO-DBL inference (forward + decode + NMS) images/sec on MI355X.

Default workload = BASELINE.json configs[1]: YOLO-DBL-n, 640x640, bs=32 per GPU,
fp16, predict settings (conf 0.25, iou 0.7, max_det 300), synthetic blob images
already resident in HBM, trained-like synthetic weights (tests/golden fixture).
A step = one hipGraph replay of forward + decode + NMS over the batch, plus (N>1)
one RCCL all-gather of the per-image [det | count] records (ydbl.parallel).

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
        "l": ("yolov13l_DBL2.yaml", "trained_yolov13l_DBL2_nc3.npz"),
        "x": ("yolov13x_DBL2.yaml", "trained_yolov13x_DBL2_nc3.npz")}


def _px(v):
    return v.n * v.h * v.w


def conv_traffic(step, elsize):
    """Algorithmic bytes / FLOPs of one ydbl_conv2d_nhwc launch from its descriptor: input read once,
    output written once (+ residual read, + fused FullPAD second output and its other input), weights once."""
    d = step.args[0]
    x, y = d.x, d.y
    cin = x.c
    k = d.kh * d.kw
    wsize = 1 if d.dq else elsize  # e4m3 weights in fp8 mode
    byts = (_px(x) * cin + _px(y) * y.c) * elsize + y.c * k * cin * wsize
    if d.res_mode:
        byts += _px(y) * y.c * elsize
    if d.y2.ptr:
        byts += 2 * _px(y) * y.c * elsize
    return byts, 2.0 * _px(y) * y.c * k * cin


def dsconv_traffic(step, elsize):
    """ydbl_dsconv_nhwc: x read, y written (+ residual, + the fused class-conv output), dw + pw weights."""
    d = step.args[0]
    x, y = d.x, d.y
    byts = (_px(x) * x.c + _px(y) * y.c) * elsize + x.c * d.k * d.k * 4 + y.c * x.c * elsize
    if d.res_mode:
        byts += _px(y) * y.c * elsize
    if d.tail_w:
        byts += _px(y) * d.tail_n * elsize
    flops = 2.0 * _px(y) * x.c * (d.k * d.k + y.c)
    if d.g2_w:  # trailing GEMM (C3's cv3): y stays on chip; the cv2 branch is read and cv3's output written
        byts += (_px(d.g2_x) * d.g2_x.c + _px(d.g2_y) * d.g2_y.c - _px(y) * y.c) * elsize
        flops += 2.0 * _px(d.g2_y) * d.g2_y.c * (y.c + d.g2_x.c)
    if d.g0_w:  # leading 1x1 (C3's cv2 | cv1): its input read and both outputs written instead of x read
        byts += (_px(d.g0_x) * d.g0_x.c + _px(d.g0_y) * d.g0_y.c - _px(x) * x.c) * elsize + d.g0_y.c * d.g0_x.c * elsize
        flops += 2.0 * _px(d.g0_y) * d.g0_y.c * d.g0_x.c
    return byts, flops


def bneck_traffic(step, elsize):
    """ydbl_bottleneck_nhwc: Conv3x3(c_in, c_mid) -> Conv3x3(c_mid, c) [-> 1x1 c -> c]: x read, y written."""
    d = step.args[0]
    x, y = d.x, d.y
    cm = d.c_mid or d.c // 2
    flops = 2.0 * _px(y) * (x.c * 9 * cm + cm * 9 * d.c + (d.c * d.c if d.pw else 0))
    return (_px(x) * x.c + _px(y) * y.c) * elsize, flops


def stem2_traffic(step, elsize):
    """ydbl_conv_stem2: the fp32 NCHW image read, layer 1's output written (layer 0's stays on chip)."""
    d = step.args[0]
    c0 = d.c0
    flops = 2.0 * d.n * d.h * d.w * c0 * 27 + 2.0 * _px(d.y) * 2 * c0 * 9 * c0
    return d.n * d.cin * d.h * d.w * 4 + _px(d.y) * d.y.c * elsize, flops


def dysample_traffic(step, elsize):
    """ydbl_dysample_ex: x + offsets read, the 2x-upsampled y written (+ fused FullPAD second output)."""
    d = step.args[0]
    byts = (_px(d.x) * d.x.c + _px(d.off) * d.off.c + _px(d.y) * d.y.c) * elsize
    if d.y2.ptr:
        byts += 2 * _px(d.y) * d.y.c * elsize
    return byts, 0.0


def _v(v):
    """(pixels, channels) of a ydbl_view struct or pointer to one (None / NULL view -> (0, 0))."""
    if v is None:
        return 0, 0
    v = getattr(v, "contents", v)
    return (_px(v), v.c) if v.ptr else (0, 0)


def views_traffic(reads, writes, elsize, flops=0.0):
    return (sum(p * c for p, c in map(_v, reads)) + sum(p * c for p, c in map(_v, writes))) * elsize, flops


def other_traffic(step, elsize):
    """Algorithmic bytes / FLOPs of the remaining launch kinds (activations read once and written
    once at the run dtype; small weights and the NMS candidate lists are left out)."""
    k, a = step.fn.__name__, step.args
    if k == "ydbl_dwconv2d_pair_nhwc":
        d0, d1 = a[0], a[1]
        return views_traffic([d0.x], [d0.y, d1.y], elsize, 2.0 * _px(d0.y) * d0.y.c * (d0.kh * d0.kw + d1.kh * d1.kw))
    if k == "ydbl_dwconv2d_nhwc":
        d = a[0]
        return views_traffic([d.x] + ([d.r] if d.res_mode else []), [d.y], elsize, 2.0 * _px(d.y) * d.y.c * d.kh * d.kw)
    if k == "ydbl_lsk_gate":
        return views_traffic([a[0]], [a[3]], elsize, 2.0 * _v(a[3])[0] * (98 * 2 + a[3].c * 2))
    if k == "ydbl_pool_up_concat":
        return views_traffic([a[0], a[1], a[2]], [a[3]], elsize)
    if k == "ydbl_gate_add":
        return views_traffic([a[0], a[1]], [a[3]], elsize)
    if k in ("ydbl_hg_context", "ydbl_hg_propagate"):
        d = a[0]
        n, dd, e = _px(d.x), d.x.c, d.num_edges
        if k == "ydbl_hg_context":
            return views_traffic([d.x], [], elsize, 2.0 * d.x.n * e * dd * 2 * dd)
        return views_traffic([d.x, d.xp], [d.y], elsize, 2.0 * n * (2 * e * dd + 2 * dd * dd))
    if k == "ydbl_conv_stem":
        n, cin, h, w, y = a[1], a[2], a[3], a[4], a[11]
        return n * cin * h * w * 4 + _v(y)[0] * y.c * elsize, 2.0 * _v(y)[0] * y.c * 27
    if k == "ydbl_detect_decode":
        d = a[0]
        reads = [d.box[i] for i in range(d.nl)] + [d.cls[i] for i in range(d.nl)]
        return views_traffic(reads, [], elsize)
    return 0.0, 0.0


def dysample2_traffic(step, elsize):
    """ydbl_dysample2: x read once (offset conv and sample), the 2x-upsampled y written (+ FullPAD second output)."""
    d = step.args[0]
    byts = (_px(d.x) * d.x.c + _px(d.y) * d.y.c) * elsize
    if d.y2.ptr:
        byts += 2 * _px(d.y) * d.y.c * elsize
    return byts, 2.0 * _px(d.x) * d.x.c * 8 * d.groups


def hg_fused_traffic(step, elsize):
    """ydbl_hg_fused: the tokens X read once, y written once (the pre_head_proj xp never leaves the CU)."""
    d = step.args[0]
    n, dd, e = _px(d.x), d.x.c, d.num_edges
    return 2 * n * dd * elsize, 2.0 * n * (dd * dd + 3 * e * dd) + 2.0 * d.x.n * e * dd * (2 * dd + 2 * dd)


def lsk_traffic(step, elsize):
    """ydbl_lsk_attn: a1, a2 read, attn = conv1(a1) | conv2(a2) written (+ per-pixel stats, left out);
    ydbl_lsk_out: attn and x read, y = x * conv(gate(attn)) written (LSKA.py:43-52)."""
    d = step.args[0]
    p, dim = _px(d.x), d.x.c
    if step.fn.__name__ == "ydbl_lsk_attn":
        return 3 * p * dim * elsize, 2.0 * p * dim * dim
    return 3 * p * dim * elsize, 2.0 * p * (dim // 2) * dim + 2.0 * p * 98 * 2


TRAFFIC = {"ydbl_conv2d_nhwc": ("conv2d", conv_traffic), "ydbl_dsconv_nhwc": ("dsconv", dsconv_traffic),
           "ydbl_dysample2": ("dysample", dysample2_traffic), "ydbl_hg_fused": ("hypergraph", hg_fused_traffic),
           "ydbl_bottleneck_nhwc": ("bottleneck", bneck_traffic), "ydbl_conv_stem2": ("stem2", stem2_traffic),
           "ydbl_dysample_ex": ("dysample", dysample_traffic), "ydbl_lsk_attn": ("lsk", lsk_traffic),
           "ydbl_lsk_out": ("lsk", lsk_traffic)}


def roofline(session, dtype_name, key=None, step_ms=None):
    """Per-launch time of every launch of every plan of the session as it runs inside a hipGraph
    (Plan.run_graph_timed: the launch captured 8x into a graph, replayed between HIP events on the
    replaying stream, min of 3 / 8 -- the figure rocprofv3 reports per kernel); the dominant kernel
    family (most time) = the dense conv; a per-family table beside it; and the whole-network figure of
    SURVEY §8d: t_k = max(bytes_k / HBM peak, flops_k / MFMA peak) per launch, sum over every launch of
    the step, divided by the measured step time `step_ms` of the timed run."""
    elsize = 4 if dtype_name == "fp32" else 2  # activation bytes (fp8 mode keeps fp16 activations)
    steps, best = [], []
    for plan in session.plans:  # one plan per sub-batch stream (each launch timed on its own)
        steps += plan.steps
        best += plan.run_graph_timed()
    by_kind, fam = {}, {}
    for st, (what, ms) in zip(steps, best):
        kind = st.fn.__name__
        by_kind[kind] = by_kind.get(kind, 0.0) + ms
        if kind in TRAFFIC:
            name, fn = TRAFFIC[kind]
            b, f = fn(st, elsize)
            e = fam.setdefault(name, {"launches": 0, "ms": 0.0, "bytes": 0.0, "flops": 0.0})
            e["launches"] += 1
            e["ms"] += ms
            e["bytes"] += b
            e["flops"] += f
    pk = MFMA_PEAK_TFLOPS[dtype_name]
    net_b = net_f = t_roof = 0.0
    for st in steps:
        kind = st.fn.__name__
        b, f = TRAFFIC[kind][1](st, elsize) if kind in TRAFFIC else other_traffic(st, elsize)
        net_b, net_f = net_b + b, net_f + f
        t_roof += max(b / (HBM_PEAK_GBS * 1e9), f / (pk * 1e12))
    launch_ms = sum(ms for _, ms in best)
    network = {"launches_per_step": len(steps), "alg_bytes_per_step": int(net_b), "alg_flops_per_step": net_f,
               "roofline_ms_per_step": round(t_roof * 1e3, 4), "sum_launch_ms_per_step": round(launch_ms, 4),
               "frac_of_sum_launch": round(t_roof * 1e3 / launch_ms, 4),
               "rule": "sum_k max(bytes_k / 8 TB/s, flops_k / MFMA peak) over every launch of the step "
                       "(algorithmic bytes: activations read + written once, weights once) / step time"}
    if step_ms:
        network.update({"measured_ms_per_step": round(step_ms, 4), "frac": round(t_roof * 1e3 / step_ms, 4)})
    pmc = pmc_summary(key)
    families = {}
    for name, e in sorted(fam.items(), key=lambda kv: -kv[1]["ms"]):
        gbs = e["bytes"] / (e["ms"] * 1e-3) / 1e9
        tf = e["flops"] / (e["ms"] * 1e-3) / 1e12
        families[name] = {"launches": e["launches"], "avg_launch_us": round(e["ms"] * 1e3 / e["launches"], 2),
                          "alg_bytes_per_launch": int(e["bytes"] / e["launches"]), "GB_s": round(gbs, 1),
                          "hbm_frac": round(gbs / HBM_PEAK_GBS, 4), "TFLOP_s": round(tf, 2),
                          "mfma_frac": round(tf / pk, 4)}
        if pmc and name in pmc["families"]:
            pf = pmc["families"][name]
            families[name]["pmc_hbm_bytes_per_launch"] = pf.get("hbm_bytes_per_launch")
            families[name]["mfma_busy"] = pf.get("mfma_busy")
    c = fam["conv2d"]
    ach_gbs = c["bytes"] / (c["ms"] * 1e-3) / 1e9
    ach_tf = c["flops"] / (c["ms"] * 1e-3) / 1e12
    ai = c["flops"] / c["bytes"]
    ridge = pk * 1e12 / (HBM_PEAK_GBS * 1e9)
    if ai < ridge:
        rf = {"bound": "hbm", "achieved": round(ach_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(ach_gbs / HBM_PEAK_GBS, 4)}
    else:
        rf = {"bound": "mfma", "achieved": round(ach_tf, 2), "peak": pk, "unit": "TFLOP/s", "frac": round(ach_tf / pk, 4)}
    pc = pmc["families"].get("conv2d", {}) if pmc else {}
    rf.update({"kernel": "ydbl_conv2d_nhwc", "launches_per_step": c["launches"],
               "avg_launch_us": round(c["ms"] * 1e3 / c["launches"], 2),
               "alg_bytes_per_launch": int(c["bytes"] / c["launches"]), "alg_flops_per_step": c["flops"],
               "arith_intensity": round(ai, 1), "tflops": round(ach_tf, 2),
               "sum_launch_ms": round(launch_ms, 3), "launch_timing": "in-graph (Plan.run_graph_timed)",
               "network": network,
               "ms_by_kernel": {k: round(v, 3) for k, v in sorted(by_kind.items(), key=lambda kv: -kv[1])},
               "traffic": pc.get("hbm_bytes_per_launch"), "mfma_busy": pc.get("mfma_busy"),
               "code_hash": code_hash(),
               "pmc_summary": pmc["file"] if pmc else "none for this code hash and workload (scripts/pmc_families.sh)",
               "families": families})
    return rf


def code_hash() -> str:
    sys.path.insert(0, str(ROOT / "scripts"))
    from pmc_summary import code_hash as ch

    return ch()


def workload_key(args, dtype_name) -> str:
    """What a PMC summary must have been measured on to describe this run's launches."""
    return f"model={args.model} batch={args.batch} imgsz={args.imgsz} dtype={dtype_name} streams={args.streams}"


def pmc_summary(key=None):
    """The newest committed profiles/*_pmc_families.json measured on THIS code (matching source hash) and,
    when `key` is given, on this workload (scripts/pmc_families.sh records bench.py's workload_key)."""
    h = code_hash()
    for p in sorted((ROOT / "profiles").rglob("*_pmc_families.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("code_hash") == h and (key is None or d.get("workload") == key):
            d["file"] = str(p.relative_to(ROOT))
            return d
    return None


def _cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(model_key, imgsz, batch, budget_s=10.0, gpu_session=None):
    """The oracle (CPU restatement of the reference path, fp32, BN folded as fuse() does) timed on this
    box's host cores over bounded samples of the same workload: forward + decode +
    NMS (conf .25, iou .7) + clip per image.
      leg 1: all intra-op threads, bs = the GPU batch (the headline `value`);
      leg 2: 1 thread (the reference's import-time OMP_NUM_THREADS=1 default, U/__init__.py:9-10), bs=1.
    Also the accuracy half of the metric: mAP@0.5 of the GPU path vs the CPU path on a fixed labelled
    set (pseudo ground truth = CPU detections at conf .25), when gpu_session is given."""
    sys.path.insert(0, str(ROOT))
    from oracle.model import build_model
    from oracle.ops import clip_boxes, non_max_suppression
    from ydbl.utils.synthetic import blob_images, load_trained

    cfg, fx = CFGS[model_key]
    torch.manual_seed(0)
    m = build_model(cfg, nc=3)
    load_trained(m, ROOT / "tests" / "golden" / fx)
    m.fuse()
    threads_all = torch.get_num_threads()

    def leg(bs, threads):
        torch.set_num_threads(threads)
        x = blob_images(bs, imgsz, seed=1234)
        with torch.inference_mode():
            def once():
                y, _ = m(x)
                for d in non_max_suppression(y, 0.25, 0.7):
                    clip_boxes(d[:, :4], (imgsz, imgsz))
            once()  # warm-up
            n, t0 = 0, time.perf_counter()
            while True:
                once()
                n += 1
                el = time.perf_counter() - t0
                if el > budget_s or n >= 50:
                    break
        return {"img_per_s": round(n * bs / el, 3), "bs": bs, "threads": threads, "iters": n, "secs": round(el, 1)}

    legs = [leg(batch, threads_all), leg(1, 1)]
    torch.set_num_threads(threads_all)
    # `cores` = the threads actually used (torch intra-op threads of this process on the box's CPU share);
    # os_cpu_count is the whole machine's logical CPUs, most of which belong to other jobs
    out = {"value": legs[0]["img_per_s"], "unit": "images/s", "cores": threads_all, "threads": threads_all,
           "cores_note": f"{threads_all} intra-op threads (= cores used) of {os.cpu_count()} logical CPUs on the host",
           "kind": "port",
           "sample": f"{legs[0]['iters']} x bs{batch} DBL-{model_key} {imgsz}x{imgsz} nc3 fp32 oracle forward+NMS "
                     f"on {threads_all} threads ({legs[0]['secs']} s); 1-thread leg: {legs[1]['img_per_s']} img/s",
           "legs": legs, "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count()}
    if gpu_session is not None:
        out["map50"] = accuracy_check(m, gpu_session, imgsz)
    return out


def accuracy_check(m, gpu, imgsz, n=8):
    """|mAP50_gpu - mAP50_cpu| on n blob images with pseudo ground truth (SURVEY §8d protocol; the same
    val pipeline -- conf .001, multi-label NMS, iou .7 -- scores both paths)."""
    from oracle.metrics import IOUV, box_iou, match_predictions
    from oracle.ops import clip_boxes, non_max_suppression
    from ydbl.utils.metrics import DetMetrics
    from ydbl.utils.synthetic import blob_images

    x = blob_images(n, imgsz, seed=321)
    with torch.inference_mode():
        y, _ = m(x)
    labels = []
    for g in non_max_suppression(y, 0.25, 0.7):
        clip_boxes(g[:, :4], (imgsz, imgsz))
        labels.append(torch.cat([g[:, 5:6], g[:, :4]], 1))
    st = {"tp": [], "conf": [], "pred_cls": [], "target_cls": []}
    for i, p in enumerate(non_max_suppression(y, 0.001, 0.7, multi_label=True)):
        clip_boxes(p[:, :4], (imgsz, imgsz))
        cls, box = labels[i][:, 0], labels[i][:, 1:]
        tp = (match_predictions(p[:, 5], cls, box_iou(box, p[:, :4]), IOUV) if len(cls) and len(p)
              else torch.zeros(len(p), 10, dtype=torch.bool))
        st["tp"].append(tp); st["conf"].append(p[:, 4]); st["pred_cls"].append(p[:, 5]); st["target_cls"].append(cls)
    dm = DetMetrics()
    dm.process(*(torch.cat(st[k]).numpy() for k in ("tp", "conf", "pred_cls", "target_cls")))
    batch = {"img": x, "cls": torch.cat([lb[:, 0] for lb in labels]), "bboxes": torch.cat([lb[:, 1:] for lb in labels]),
             "batch_idx": torch.cat([torch.full((len(lb),), i) for i, lb in enumerate(labels)])}
    yolo, fp8, half = gpu  # the product YOLO (HIP path), e4m3 operands or not, fp16 or fp32 (the timed path)
    m_gpu = yolo.val(data=[batch], half=half, fp8=fp8).box.map50
    return {"gpu": round(float(m_gpu), 4), "cpu": round(float(dm.box.map50), 4),
            "drop": round(float(dm.box.map50 - m_gpu), 4),
            "images": n, "gt_boxes": int(sum(len(lb) for lb in labels)),
            "gpu_precision": "fp8" if fp8 else ("fp16" if half else "fp32"),
            "protocol": "pseudo-GT = CPU oracle detections at conf .25; val NMS conf .001 multi-label iou .7"}


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without an external launcher: run this script under torch.distributed.run as a
    CHILD process (one rank per GPU) and return its exit code.  The parent never touches the GPU (only
    `import torch`, which does not initialise HIP), so no GPU-holding process is ever replaced by exec.
    Same role as the reference's DDP launcher, U/utils/dist.py:25-66 (there: a temp script + torchrun)."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this driver
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()), *argv]
    return subprocess.call(cmd, env=env)


def stub_step_factory(B: int, world: int, rank: int):
    """--stub-cpu: the multi-rank plumbing of a step (gloo, CPU) without a GPU -- each rank fills its
    record buffer (ydbl.parallel: [det | count] per image) and takes part in the one all-gather into a
    preallocated global buffer.  Used by tests/test_bench_launch.py."""
    from ydbl.parallel import GlobalDetections, gather_records, record_views, record_width

    rec = torch.zeros(B, record_width(300))
    det, cnt = record_views(rec, 300)
    det.fill_(float(rank))
    cnt.fill_(rank + 1)
    out = torch.empty(world * B, rec.shape[1])
    glob = GlobalDetections(out, B * world, world, 300)

    def step():
        if world > 1:
            gather_records(rec, out)
            d, c = glob.tensors()
            assert d.shape[0] == B * world and int(c[-1]) == world and float(d[-1, 0, 0]) == world - 1

    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="n", choices=list(CFGS))
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--fp8", nargs="?", type=float, const=1.0, default=0.0, metavar="FRACTION",
                    help="e4m3 dense-conv operands (BASELINE config 5); FRACTION < 1 switches that share of the "
                         "candidate MACs, least output-sensitive convs first (ydbl.quant.enable_fp8)")
    ap.add_argument("--streams", type=int, default=2,
                    help="sub-batch plans run concurrently, as branches of one hipGraph (DetectSession); "
                         "2 measured +3 %% DBL-n bs32, +9 %% DBL-s bs64, +8.5 %% DBL-l 1280 bs8 over 1 (4: -33 %% DBL-n)")
    ap.add_argument("--via-predict", action="store_true",
                    help="time the public API instead of the session: each step is YOLO.predict(batch, half=...) on "
                         "the HBM-resident batch (LoadTensor checks + copy into the session's input buffer, the "
                         "same split hipGraph, the per-batch count sync, Results objects); no roofline / CPU legs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--stub-cpu", action="store_true", help="gloo/CPU plumbing check of the N-rank launch (no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the launcher started {world} ranks")
    if args.stub_cpu:
        return stub_main(args, world, rank)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        assert dist.get_world_size() == args.gpus
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
    fp8 = True if args.fp8 >= 1.0 else (args.fp8 if args.fp8 > 0 else False)
    from ydbl.parallel import ShardedPredictor

    # this rank's B images of the global batch B * world; its NMS writes the per-image [det | count] records
    # that the step's one all-gather ships (ydbl.parallel; no process group at N = 1: no collective)
    if args.via_predict:
        return predict_main(args, model, world, rank, dev, half, fp8, dtype_name, cfg)
    sp = ShardedPredictor(model, B * world, S, S, dev, half=half, conf=0.25, iou=0.7, max_det=300, fp8=fp8,
                          streams=args.streams)
    sess = sp.session
    fp8_cal = fp8_calibration_file(cfg)
    if args.fp8:  # the committed calibration of these weights (one layer set per share), else a calibration batch
        if fp8_cal is not None:
            sess.calibrate_fp8(calibration=fp8_cal)
        else:
            sess.calibrate_fp8(blob_images(B, S, seed=4321 + rank).to(dev))
    # synthetic images, different per rank, resident in the session's input buffer (HBM)
    sp.load(images_local=blob_images(B, S, seed=1234 + rank).to(dev))

    def step():
        sp.run()  # forward + decode + NMS (one hipGraph replay, the sub-batch plans as its branches) [+ the one all-gather]

    el = timed_steps(step, args, world, lambda: torch.cuda.synchronize(dev), dev)
    key = workload_key(args, dtype_name)
    if rank == 0 and os.environ.get("YDBL_WORKLOAD_KEY_OUT"):  # scripts/pmc_families.sh
        Path(os.environ["YDBL_WORKLOAD_KEY_OUT"]).write_text(key)
    extra = {"dets_per_image": round(float(sess.count.float().mean().item()), 2),
             "candidates_per_image": round(float(sess.cand_count.float().mean().item()), 1),
             "candidates_max": int(sess.cand_count.max().item())}
    if args.fp8:  # achieved share of the candidate MACs in e4m3 (output-pixel MACs, ydbl.quant.candidate_macs)
        extra["fp8_mac_fraction"] = round(float(sess.fp8_mac_fraction), 4)
    rf = None
    if rank == 0 and not args.no_roofline:
        # The roofline describes the kernels at the headline launch size: one launch per layer over the
        # whole per-GPU batch.  With --streams k the timed run splits that batch into k concurrent
        # sub-batch graphs, whose launches overlap; the per-launch view is taken on the full-batch plan.
        rsess, rkey = sess, key
        if args.streams > 1:
            rsess = model.session(B, S, S, half=half, conf=0.25, iou=0.7, max_det=300, device=dev, fp8=fp8, streams=1)
            if args.fp8 and fp8_cal is not None:
                rsess.calibrate_fp8(calibration=fp8_cal)
            elif args.fp8:
                rsess.calibrate_fp8(blob_images(B, S, seed=4321 + rank).to(dev))
            rsess.load(blob_images(B, S, seed=1234 + rank).to(dev))
            rsess()
            rkey = key.replace(f"streams={args.streams}", "streams=1")
        rf = roofline(rsess, dtype_name, key=rkey, step_ms=el * 1e3 / args.steps)
        rf["plan"] = f"full-batch plan (bs {B}, one launch per layer); timed run on {args.streams} stream(s)"
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.model, S, B, gpu_session=(model, fp8, half))
    if rank == 0:
        emit_line(args, world, el, dtype_name, cfg, extra, rf, cpu)
    if world > 1:
        dist.destroy_process_group()


def fp8_calibration_file(cfg):
    """The committed fp8 calibration of the fixture weights of `cfg` (scripts/fp8_calibrate.py), if any."""
    f = ROOT / "tests" / "golden" / f"fp8_calib_{Path(cfg).stem}_nc3.json"
    return str(f) if f.exists() else None


def predict_main(args, model, world, rank, dev, half, fp8, dtype_name, cfg):
    """--via-predict: the step is the user-facing call YOLO.predict(x, half=...) on this rank's HBM-resident
    batch, with predict()'s own stream layout (ydbl.engine.session.default_streams: the split hipGraph from
    batch 4 up); the line says so in config.via."""
    from ydbl.utils.synthetic import blob_images

    B, S = args.batch, args.imgsz
    x = blob_images(B, S, seed=1234 + rank).to(dev)
    kw = dict(half=half, fp8=fp8, conf=0.25, iou=0.7, max_det=300, device=dev, fp8_calibration=fp8_calibration_file(cfg))
    if fp8 and kw["fp8_calibration"] is None:  # calibrate once on the separate synthetic batch, as the session bench
        from ydbl.engine.session import default_streams

        model.session(B, S, S, half=True, conf=0.25, iou=0.7, max_det=300, device=dev, fp8=fp8,
                      streams=default_streams(B)).calibrate_fp8(blob_images(B, S, seed=4321 + rank).to(dev))
    out = {}

    def step():
        out["r"] = model.predict(x, **kw)

    el = timed_steps(step, args, world, lambda: torch.cuda.synchronize(dev), dev)
    if rank == 0:
        extra = {"dets_per_image": round(sum(len(r.boxes.data) for r in out["r"]) / B, 2),
                 "via": "YOLO.predict(x, half=%s) per step (Results construction included; the detections are read "
                        "back when first accessed, after the timed steps)" % half}
        emit_line(args, world, el, dtype_name, cfg, extra, None, None)
    if world > 1:
        dist.destroy_process_group()


def timed_steps(step, args, world, sync, dev=None) -> float:
    """W untimed warmup steps, then exactly K steps bracketed by barrier + device sync on both sides;
    returns the MAX over ranks of the timed wall clock (seconds)."""
    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    return el


def emit_line(args, world, el, dtype_name, cfg, extra, rf, cpu):
    B, S = args.batch, args.imgsz
    out = {
        "metric": "images/sec @640×640 bs=32 (1/2/4/8 GPU) + mAP@0.5 vs CPU ref",
        "value": round(B * world * args.steps / el, 2),
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
                   "parallelism": f"dp{world}", "streams_per_gpu": args.streams,
                   **({"fp8_mac_fraction": extra.pop("fp8_mac_fraction", None)} if args.fp8 else {})},
        **extra,
        "roofline": rf,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)


def stub_main(args, world, rank):
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus
    step = stub_step_factory(args.batch, world, rank)
    el = timed_steps(step, args, world, lambda: None)
    if rank == 0:
        emit_line(args, world, el, "stub", CFGS[args.model][0], {"stub": "gloo/CPU plumbing, no GPU work"}, None, None)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
