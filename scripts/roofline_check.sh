#!/bin/bash
# bench.py's in-graph per-launch timing vs rocprofv3's kernel durations on the same single-stream command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=gpurun_out/${1:-rfchk}; mkdir -p $T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_s1 -o run -- python bench.py --streams 1 --steps 20 --warmup 5 \
    --no-cpu-baseline > $T/prof_s1.log 2>&1 || { echo "single-stream rocprof failed"; tail -20 $T/prof_s1.log; exit 1; }
python scripts/rocpd_stats.py $T/prof_s1/run_results.db > $T/c2_streams1_kernel_stats.csv
python scripts/rocprof_families.py $T/c2_streams1_kernel_stats.csv $T/prof_s1.log
