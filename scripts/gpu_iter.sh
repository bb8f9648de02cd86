#!/bin/bash
# Kernel iteration pass on the GPU box: selected parity tests, per-launch profile, short bench.
# Usage: bash scripts/gpu_iter.sh TAG "pytest -k expression" [layer_profile args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-iter}; KEXPR=${2:-""}; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "$KEXPR" > $OUT/pytest.log 2>&1
  rc=$?; tail -4 $OUT/pytest.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; exit $rc; }
fi
timeout -k 10 300 python -u scripts/layer_profile.py "$@" > $OUT/layers.txt 2>&1 || { tail -20 $OUT/layers.txt; exit 5; }
head -16 $OUT/layers.txt
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 6; }
tail -1 $OUT/bench.log | cut -c1-400
