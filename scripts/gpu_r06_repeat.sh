#!/bin/bash
# Round 6: the default bench line as the driver runs it (roofline + PMC traffic on this code + CPU leg), then two more
# session lines and two predict() lines alternating on the same box (spread within a box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_repeat; mkdir -p $T
set -o pipefail
timeout -k 10 300 python bench.py > $T/bench_default.log 2>&1 || { tail -20 $T/bench_default.log; exit 1; }
tail -1 $T/bench_default.log > $T/bench_default.json
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['frac'], r['traffic'], r['mfma_busy'], r['pmc_summary'])" $T/bench_default.json
for r in 1 2; do
  for m in session predict; do
    A=""; [ $m = predict ] && A="--via-predict"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $A > $T/b_${m}_$r.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $T/b_${m}_$r.log "$m r$r"
  done
done
