#!/bin/bash
# Round-3 records on one MI355X: BASELINE configs 2-5 (bench line + rocprofv3 stats each), the PMC family summary
# of the bench workload, and a single-stream full-batch rocprofv3 summary of the bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=gpurun_out/${1:-r03rec}; mkdir -p $T
bash scripts/gpu_configs.sh ${1:-r03rec} || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_s1 -o run -- python bench.py --streams 1 --steps 20 --warmup 5 \
    --no-cpu-baseline > $T/prof_s1.log 2>&1 || { echo "single-stream rocprof failed"; tail -20 $T/prof_s1.log; exit 1; }
python scripts/rocpd_stats.py $T/prof_s1/run_results.db > $T/c2_streams1_kernel_stats.csv
tail -1 $T/prof_s1.log | cut -c1-200
bash scripts/pmc_families.sh ${1:-r03rec}_pmc $T/r03_pmc_families.json --streams 1
