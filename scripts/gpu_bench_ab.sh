#!/bin/bash
# GPU pass: selected tests (pytest -k), then bench lines for each extra-args variant.
# Usage: bash scripts/gpu_bench_ab.sh TAG "kexpr" "--streams 1" "--streams 2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; KEXPR=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "$KEXPR" > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; exit $rc; }
fi
i=0
for V in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline $V > $OUT/bench$i.log 2>&1 || { tail -20 $OUT/bench$i.log; exit 6; }
  echo "[$V] $(tail -1 $OUT/bench$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"] if d["roofline"] else None)')"
done
