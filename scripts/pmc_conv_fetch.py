"""Which conv launches fetch more HBM bytes than they algorithmically need?

Mode 1 (under rocprofv3 --pmc FETCH_SIZE, then again WRITE_SIZE): every ydbl_conv2d_nhwc step of the bench's full-batch
plan (DBL-n bs32 640 fp16, one plan) is run REPS times in a row on its own, in plan order, after one warm pass of the
whole plan (so each conv's input was just written by its producer, as in the step).  A JSON list of the steps
(order, shape, algorithmic bytes) is written next to the profile.

    python scripts/pmc_conv_fetch.py run OUT.json
    python scripts/pmc_conv_fetch.py report OUT.json FETCH_DIR WRITE_DIR      (FETCH_SIZE x2, MI355X_MICROARCH.md)
"""
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-dbl_amd")]

REPS = 5


def run(out):
    import torch

    from bench import CFGS, conv_traffic
    from ydbl import YOLO
    from ydbl.utils.synthetic import blob_images, load_trained

    cfg, fx = CFGS["n"]
    torch.manual_seed(0)
    m = YOLO(cfg, nc=3)
    load_trained(m.model, ROOT / "tests" / "golden" / fx)
    s = m.session(32, 640, 640, half=True, use_graph=False)
    s.load(blob_images(32, 640, seed=1234).cuda())
    plan = s.plan
    steps = []
    for i, st in enumerate(plan.steps):
        if st.fn.__name__ != "ydbl_conv2d_nhwc":
            continue
        d = st.args[0]
        byts, flops = conv_traffic(st, 2)
        steps.append({"step": i, "what": st.what, "cin": d.x.c, "cout": d.y.c, "k": d.kh, "s": d.stride,
                      "h": d.x.h, "w": d.x.w, "ho": d.y.h, "wo": d.y.w, "alg_bytes": byts})
    plan.run()  # warm: every buffer written once
    torch.cuda.synchronize()
    import ctypes as C

    cs = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for e in steps:
        st = plan.steps[e["step"]]
        for _ in range(REPS):
            st.fn(*st.args, cs)
        torch.cuda.synchronize()
    Path(out).write_text(json.dumps({"reps": REPS, "steps": steps}, indent=1))


def report(out, fdir, wdir):
    meta = json.loads(Path(out).read_text())
    steps, reps = meta["steps"], meta["reps"]

    def conv_dispatches(d, counter):
        rows = []
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == counter and "ydbl" in r["Kernel_Name"]:
                    rows.append((int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))), r["Kernel_Name"],
                                 float(r["Counter_Value"])))
        rows.sort()
        return rows[-len(steps) * reps:]  # the per-step repeats follow the warm pass

    fr, wr = conv_dispatches(fdir, "FETCH_SIZE"), conv_dispatches(wdir, "WRITE_SIZE")
    tot_alg = tot_pmc = 0.0
    print(f"{'step':>4} {'layer':28s} {'shape':30s} {'alg MB':>8} {'PMC MB':>8} {'ratio':>6}  kernel")
    for n, e in enumerate(steps):
        f = sum(v for _, _, v in fr[n * reps:(n + 1) * reps]) / reps
        w = sum(v for _, _, v in wr[n * reps:(n + 1) * reps]) / reps
        pmc = (2 * f + w) * 1024
        tot_alg += e["alg_bytes"]
        tot_pmc += pmc
        kname = fr[n * reps][1].split("(")[0][-50:]
        shape = f"{e['cin']}->{e['cout']} k{e['k']}s{e['s']} @{e['h']}x{e['w']}"
        print(f"{e['step']:4d} {e['what'][:28]:28s} {shape:30s} {e['alg_bytes'] / 1e6:8.2f} {pmc / 1e6:8.2f} "
              f"{pmc / e['alg_bytes']:6.2f}  {kname}")
    print(f"conv2d family: algorithmic {tot_alg / 1e6:.1f} MB, PMC {tot_pmc / 1e6:.1f} MB, ratio {tot_pmc / tot_alg:.3f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        report(*sys.argv[2:5])
