#!/bin/bash
# Round 6: NMS timing only (scripts/nms_wide_bench.py + per-kernel rocprof of three cases).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=gpurun_out/r06_nms; mkdir -p $T; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 200 python -u scripts/nms_wide_bench.py > $T/nms_wide_bench.txt 2>&1 || exit 1
for c in 0 3 6; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $T/p$c -o run -- python scripts/nms_wide_bench.py $c 1 1 \
      > $T/p$c.log 2>&1 || exit 1
  python scripts/rocpd_stats.py $T/p$c/run_results.db > $T/case${c}_kernel_stats.csv || exit 1
done
