"""Per-family kernel time from a rocprofv3 --stats kernel summary, for checking bench.py's roofline.

    python scripts/rocprof_families.py profiles/r03/c2_streams1_kernel_stats.csv [bench_line.json]

Groups the summary's kernels into the families of scripts/pmc_summary.py (conv2d = every kernel
ydbl_conv2d_nhwc dispatches) and prints kernel calls, total time and the average duration per entry-point launch of each family.  Given a bench
JSON line it also prints the line's roofline.families[*].avg_launch_us beside the rocprof average and
their ratio: the per-launch in-graph timing of bench.py must agree within 5 %.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import family  # noqa: E402

KERNELS_PER_LAUNCH = {"hypergraph": 5}  # ydbl_hg_fused: ctx, proto, edge, merge, out kernels per entry-point call


def families(path):
    out = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        fam = family(r["Name"])
        if fam:
            out[fam][0] += int(r["Calls"])
            out[fam][1] += float(r["TotalDurationNs"])
    res = {}
    for k, (c, t) in out.items():
        launches = c / KERNELS_PER_LAUNCH.get(k, 1)
        res[k] = {"calls": c, "total_ms": round(t / 1e6, 3), "avg_us": round(t / launches / 1e3, 2)}
    return res


def main():
    fams = families(sys.argv[1])
    line = None
    if len(sys.argv) > 2:
        txt = Path(sys.argv[2]).read_text().strip().splitlines()
        line = json.loads([t for t in txt if t.startswith("{")][-1])
    bf = (line or {}).get("roofline", {}).get("families", {})
    for k, v in sorted(fams.items(), key=lambda kv: -kv[1]["total_ms"]):
        s = f"{k:12s} calls {v['calls']:6d}  total {v['total_ms']:9.3f} ms  avg {v['avg_us']:8.2f} us"
        if k in bf:
            b = bf[k]["avg_launch_us"]
            s += f"   bench {b:8.2f} us  bench/rocprof {b / v['avg_us']:.3f}"
        print(s)


if __name__ == "__main__":
    main()
