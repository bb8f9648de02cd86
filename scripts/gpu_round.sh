#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel trace of the bench.
# Usage (from the repo root, on the GPU box): bash scripts/gpu_round.sh [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a $OUT/pytest_gpu.log; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { echo "GPU parity tests FAILED (rc=$rc): not running smoke/bench/profile"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 3; }
tail -3 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -30 $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo prof failed; tail -30 $OUT/prof.log; exit 5; }
find $OUT/prof -name '*stats*' | head
