#!/bin/bash
# BASELINE configs 2-5 on one MI355X: one bench.py JSON line each + a rocprofv3 --kernel-trace --stats summary of
# the same command (tag = $1, part $2 = 1 or 2; copy the results into profiles/<round>/ afterwards).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=gpurun_out/${1:-cfg}; mkdir -p $T; export TMPDIR=/tmp
set -o pipefail
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $T/$n.json.log 2>&1 || { echo "bench $n failed"; tail -20 $T/$n.json.log; exit 1; }
  tail -1 $T/$n.json.log > $T/$n.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_$n -o run -- python bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline --no-roofline "$@" > $T/prof_$n.log 2>&1 || { echo "rocprof $n failed"; tail -20 $T/prof_$n.log; exit 1; }
  python scripts/rocpd_stats.py $T/prof_$n/run_results.db > $T/${n}_kernel_stats.csv
  echo "$n: $(cut -c1-160 $T/$n.json)"
}
if [ "${2:-1}" = 1 ]; then
  run c2_dbl_n_bs32_fp16 --model n
  run c2_dbl_n_bs32_fp16_via_predict --model n --via-predict --no-cpu-baseline
  run c3_dbl_s_bs8_per_rank --model s --batch 8 --no-cpu-baseline
  run c3_dbl_s_bs64_fp16 --model s --batch 64 --no-cpu-baseline
else
  run c4_dbl_l_1280_bs8_fp16 --model l --batch 8 --imgsz 1280 --steps 20 --warmup 5 --no-cpu-baseline
  run c5_dbl_s_bs32_fp8_10pct --model s --fp8 0.1 --no-cpu-baseline
  run c5_dbl_s_bs32_fp8mixed25 --model s --fp8 0.25 --no-cpu-baseline
  run c5_dbl_s_bs32_fp8 --model s --fp8 --no-cpu-baseline
  run c5_dbl_s_bs32_fp16 --model s --no-cpu-baseline
fi
