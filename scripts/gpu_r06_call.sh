#!/bin/bash
# Round 6 combined call: NMS parity + timing, stem2 nontemporal A/B, bench + rocprof of configs 2 and 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
set -o pipefail
bash scripts/gpu_r06_nms.sh || { echo "nms step failed"; exit 1; }
bash scripts/gpu_lib_ab.sh r06_stem2nt "stem2" > gpurun_out/r06_stem2nt.txt 2>&1 || { echo "stem2 ab failed"; exit 1; }
T=gpurun_out/r06_cfg; mkdir -p $T
for cfg in "c2:--model n" "c3:--model s --batch 8"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $T/$n.json.log 2>&1 || { echo "bench $n failed"; exit 1; }
  tail -1 $T/$n.json.log > $T/$n.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_$n -o run -- python bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline --no-roofline $a > $T/prof_$n.log 2>&1 || { echo "rocprof $n failed"; exit 1; }
  python scripts/rocpd_stats.py $T/prof_$n/run_results.db > $T/${n}_kernel_stats.csv
done
