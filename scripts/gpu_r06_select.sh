#!/bin/bash
# Round 6: NMS above 8192 candidates by radix select + bucket sorts (nms_select_sort): parity, ydbl_nms timing
# (scripts/nms_wide_bench.py, the pair-matrix rows must be unchanged), val() at conf 0.001 on DBL-l 1280 nc80.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_select; mkdir -p $T
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread \
    -k "nms" > $T/pytest_nms.txt 2>&1 || { tail -30 $T/pytest_nms.txt; exit 1; }
tail -1 $T/pytest_nms.txt
timeout -k 10 300 python -u scripts/nms_wide_bench.py > $T/nms_wide_bench.txt 2>&1 || { tail -20 $T/nms_wide_bench.txt; exit 1; }
grep -v amdgpu $T/nms_wide_bench.txt
timeout -k 10 400 python -u scripts/val_timing.py > $T/val_timing.txt 2>&1 || { tail -20 $T/val_timing.txt; exit 1; }
tail -6 $T/val_timing.txt
