#!/bin/bash
# in-graph layer profile of the bs16 sub-batch plan, then the round-3 records (scripts/gpu_r03_all.sh) and the
# bench-vs-rocprof family check on the single-stream summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=gpurun_out/${1:-r03fin}; mkdir -p $T
timeout -k 10 200 python scripts/layer_profile.py --batch 16 > $T/layer_profile_n_bs16.txt 2>&1 || { tail $T/layer_profile_n_bs16.txt; exit 1; }
head -3 $T/layer_profile_n_bs16.txt
bash scripts/gpu_r03_all.sh ${1:-r03fin} || exit 1
python scripts/rocprof_families.py $T/c2_streams1_kernel_stats.csv $T/prof_s1.log
