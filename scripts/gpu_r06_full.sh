#!/bin/bash
# Round 6: the full GPU suite, then bench lines + rocprofv3 summaries of configs 2 (session and predict), 3 and 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_full; mkdir -p $T
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $T/pytest_gpu.txt 2>&1 \
    || { tail -40 $T/pytest_gpu.txt; exit 1; }
tail -2 $T/pytest_gpu.txt
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $T/$n.json.log 2>&1 || { echo "bench $n failed"; tail -20 $T/$n.json.log; exit 1; }
  tail -1 $T/$n.json.log > $T/$n.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_$n -o run -- python bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline --no-roofline "$@" > $T/prof_$n.log 2>&1 || { echo "rocprof $n failed"; tail -20 $T/prof_$n.log; exit 1; }
  python scripts/rocpd_stats.py $T/prof_$n/run_results.db > $T/${n}_kernel_stats.csv
  echo "$n: $(cut -c1-200 $T/$n.json)"
}
run c2_dbl_n_bs32_fp16 --model n
run c2_dbl_n_bs32_fp16_via_predict --model n --via-predict --no-cpu-baseline
run c3_dbl_s_bs8_per_rank --model s --batch 8 --no-cpu-baseline
run c4_dbl_l_1280_bs8_fp16 --model l --batch 8 --imgsz 1280 --steps 20 --warmup 5 --no-cpu-baseline
