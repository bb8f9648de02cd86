#!/bin/bash
# Round 6: wide pair-matrix NMS -- bit-exactness tests, then the on/off timing (scripts/nms_wide_bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=gpurun_out/r06_nms; mkdir -p $T; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
    -k "nms" > $T/pytest_nms.txt 2>&1 &&
timeout -k 10 200 python -u scripts/nms_wide_bench.py > $T/nms_wide_bench.txt 2>&1
