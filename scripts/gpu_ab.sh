#!/bin/bash
# Focused GPU pass: selected parity tests (-k EXPR), then bench.py (+ optional extra bench args) on the current tree.
# Usage (GPU box, repo root): bash scripts/gpu_ab.sh TAG "pytest -k expr" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/bench.log 2>&1 || { echo bench failed; tail -20 $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['roofline'].get('network',{}).get('launches_per_step'))"
