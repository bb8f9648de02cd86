#!/bin/bash
# PMC passes over the bench workload (one counter group per rocprofv3 run, --kernel-trace only, each
# under its own timeout; MI355X_MICROARCH.md rocprofv3 section) + a --stats kernel trace, then the
# per-family summary.  Usage on the GPU box: bash scripts/pmc_families.sh TAG OUT_JSON [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; OUTJ=$2; shift 2
T=gpurun_out/$TAG; mkdir -p $T; export TMPDIR=/tmp
BENCH="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline $*"
YDBL_WORKLOAD_KEY_OUT=$T/workload.txt timeout -k 10 120 $BENCH > $T/key.log 2>&1 || { echo "bench failed"; tail -5 $T/key.log; exit 1; }
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -f csv -d $T/p$i -o run -- $BENCH > $T/p$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -5 $T/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $T $OUTJ "$(cat $T/workload.txt)" > $T/summary.txt && head -40 $T/summary.txt
