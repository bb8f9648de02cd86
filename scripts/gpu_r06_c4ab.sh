#!/bin/bash
# Round 6: config 4 (DBL-l 1280 bs8, two bs4 graphs) split-K on / off: same-process A/B + rocprof with it off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_c4ab; mkdir -p $T
set -o pipefail
timeout -k 10 400 python -u scripts/ab_bench.py "split:" "nosplit:YDBL_SPLITK=0" --model l --batch 8 --imgsz 1280 \
    --rounds 3 --steps 10 > $T/ab_l8.txt 2>&1 || exit 1
YDBL_SPLITK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_off -o run -- python bench.py --steps 20 \
    --warmup 5 --no-cpu-baseline --no-roofline --model l --batch 8 --imgsz 1280 > $T/prof_off.log 2>&1 || exit 1
python scripts/rocpd_stats.py $T/prof_off/run_results.db > $T/c4_off_kernel_stats.csv
