#!/bin/bash
# Round 6: wide pair-matrix NMS -- bit-exactness tests, then the on/off timing (scripts/nms_wide_bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=gpurun_out/r06_nms; mkdir -p $T; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
    -k "nms" > $T/pytest_nms.txt 2>&1 && timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "nms or predict or split" > $T/pytest_model.txt 2>&1 &&
timeout -k 10 200 python -u scripts/nms_wide_bench.py > $T/nms_wide_bench.txt 2>&1
timeout -k 10 120 python -u scripts/nms_wide_stamps.py > $T/stamps.txt 2>&1
for c in 0 3 6; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $T/p$c -o run -- python scripts/nms_wide_bench.py $c 1 1 \
      > $T/p$c.log 2>&1 || exit 1
  python scripts/rocpd_stats.py $T/p$c/run_results.db > $T/case${c}_kernel_stats.csv || exit 1
done
