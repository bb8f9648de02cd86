#!/bin/bash
# Round-4 records, part $2 (1: parity printouts + layer profile + configs 2-5; 2: config-3 per-rank workload,
# single-stream rocprof summary, PMC families).  Copy the results into profiles/r04/ afterwards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=gpurun_out/${1:-r04rec}; mkdir -p $T
if [ "${2:-1}" = 1 ]; then
  timeout -k 10 200 python scripts/layer_profile.py --batch 16 > $T/layers_dbl_n_bs16.txt 2>&1 || { tail $T/layers_dbl_n_bs16.txt; exit 1; }
  head -2 $T/layers_dbl_n_bs16.txt | tail -1
  timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_model.py -x -q -s --timeout 300 --timeout-method thread \
      -p no:cacheprovider -k "e2e or map50_config5" > $T/e2e_fp8_tests.log 2>&1; rc=$?
  grep -E "fp32:|fp16|gpu - oracle|mAP50|s640 bs32 fp8|passed|failed" $T/e2e_fp8_tests.log | cut -c1-220 | tail -40; [ $rc -eq 0 ] || exit $rc
  bash scripts/gpu_configs.sh ${1:-r04rec} || exit 1
else
  timeout -k 10 200 python scripts/layer_profile.py --batch 32 > $T/layers_dbl_n_bs32.txt 2>&1 || { tail $T/layers_dbl_n_bs32.txt; exit 1; }
  head -2 $T/layers_dbl_n_bs32.txt | tail -1
  timeout -k 10 300 python bench.py --model s --batch 8 --no-cpu-baseline > $T/c3_dbl_s_bs8_per_rank.json.log 2>&1 || { tail $T/c3_dbl_s_bs8_per_rank.json.log; exit 1; }
  tail -1 $T/c3_dbl_s_bs8_per_rank.json.log > $T/c3_dbl_s_bs8_per_rank.json; cut -c1-200 $T/c3_dbl_s_bs8_per_rank.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_s1 -o run -- python bench.py --streams 1 --steps 20 --warmup 5 \
      --no-cpu-baseline > $T/prof_s1.log 2>&1 || { echo "single-stream rocprof failed"; tail -20 $T/prof_s1.log; exit 1; }
  python scripts/rocpd_stats.py $T/prof_s1/run_results.db > $T/c2_streams1_kernel_stats.csv
  grep "^{\"metric\"" $T/prof_s1.log | tail -1 > $T/c2_streams1_bench.json
  python scripts/rocprof_families.py $T/c2_streams1_kernel_stats.csv $T/c2_streams1_bench.json > $T/roofline_vs_rocprof.txt 2>&1; cat $T/roofline_vs_rocprof.txt | head -20
  bash scripts/pmc_families.sh ${1:-r04rec}_pmc $T/r04_pmc_families.json --streams 1
fi
