# NMS kernel durations per candidate count (rocprofv3 kernel trace over scripts/nms_bench.py); tag = $1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=gpurun_out/${1:-nmsp}; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $T -o nms -- python scripts/nms_bench.py > $T/nms.txt 2>&1 || exit 1
python - $T/nms_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "nms_kernel" in r["Kernel_Name"]]
for i, n in enumerate((0, 50, 400, 2000, 8000)):
    seg = sorted(d[13 * i:13 * i + 13])
    print(f"cands/img {n:5d}: nms_kernel median {seg[len(seg) // 2]:7.1f} us")
PY
