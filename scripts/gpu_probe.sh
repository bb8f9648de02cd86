#!/bin/bash
# GPU pass: full parity suite, then the end-to-end deviation probe at the BASELINE shapes, then a bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-probe}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 400 python -u scripts/parity_probe.py > $OUT/probe.log 2>&1 || { tail -30 $OUT/probe.log; exit 7; }
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 6; }
tail -1 $OUT/bench.log | cut -c1-600
