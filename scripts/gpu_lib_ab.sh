# Same-box A/B of two builds of libydbl.so: the in-tree library vs ${BASE:-ab_base/libydbl_base.so} (YDBL_LIB), over
set -o pipefail
# scripts/kbench.py shapes (filters as arguments) and bench.py DBL-n bs32, twice each, alternating; plus the
# GPU parity tests named by $PARITY (pytest -k expression) on the in-tree library first.
# usage: PARITY="stem2 or bottleneck" bash scripts/gpu_lib_ab.sh TAG "kbench filter" ...
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
if [ -n "$PARITY" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k "$PARITY" -x -q --timeout 120 --timeout-method thread \
    > $T/parity.log 2>&1 || { tail -30 $T/parity.log; exit 1; }
  tail -1 $T/parity.log
fi
for r in 1 2; do
  for v in base new; do
    L=""; [ $v = base ] && L="YDBL_LIB=${BASE:-ab_base/libydbl_base.so}"
    for f in "$@"; do
      env $L timeout -k 10 200 python scripts/kbench.py "$f" 2>&1 | grep "us/launch" | sed "s/^/$v r$r: /" || exit 1
    done
  done
done
# VIA_PREDICT=1: also bench.py --via-predict (the public predict() on the resident batch)
MODES="session"; [ -n "$VIA_PREDICT" ] && MODES="session predict"
for m in $MODES; do
  A=""; [ $m = predict ] && A="--via-predict"
  for r in 1 2; do
    for v in base new; do
      L=""; [ $v = base ] && L="YDBL_LIB=${BASE:-ab_base/libydbl_base.so}"
      env $L timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $A > $T/bench_${m}_${v}_r$r.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $T/bench_${m}_${v}_r$r.json "bench $m $v r$r"
    done
  done
done
