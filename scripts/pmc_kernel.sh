#!/bin/bash
# SQ counter passes over one command (kernel-trace only, one pass per counter group; MI355X_MICROARCH.md
# rocprofv3 PMC section).  Usage: bash scripts/pmc_kernel.sh TAG -- python scripts/conv_bench.py 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift; [ "$1" = "--" ] && shift
T=gpurun_out/$TAG; mkdir -p $T; export TMPDIR=/tmp
[ -f gpurun_out/counters_list.txt ] || rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -f csv -d $T/p$i -o run -- "$@" > $T/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $T/p$i.log; exit 1; }
done
python - "$T" <<'PY'
import csv, glob, sys, collections
t = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(f"{t}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:16.0f}")
PY
