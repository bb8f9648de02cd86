# Round 5: PMC families on the final source hash for the roofline's workload (bench.py --streams 1: the full-batch
# plan whose per-launch view the bench line reports; the workload key names the streams), the single-stream
# rocprofv3 summary of the bench command checked against the bench's per-launch times, and the layer profile.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05pmc; mkdir -p $T
set -o pipefail
bash scripts/pmc_families.sh r05pmc_fam $T/r05_pmc_families.json --streams 1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof_s1 -o run -- python bench.py --streams 1 --steps 20 --warmup 5 \
    --no-cpu-baseline > $T/prof_s1.log 2>&1 || { echo "single-stream rocprof failed"; tail -20 $T/prof_s1.log; exit 1; }
python scripts/rocpd_stats.py $T/prof_s1/run_results.db > $T/c2_streams1_kernel_stats.csv
grep "^{\"metric\"" $T/prof_s1.log | tail -1 > $T/c2_streams1_bench.json
python scripts/rocprof_families.py $T/c2_streams1_kernel_stats.csv $T/c2_streams1_bench.json > $T/roofline_vs_rocprof.txt 2>&1; head -20 $T/roofline_vs_rocprof.txt
timeout -k 10 200 python scripts/layer_profile.py --batch 16 > $T/layers_dbl_n_bs16.txt 2>&1 || { tail $T/layers_dbl_n_bs16.txt; exit 1; }
timeout -k 10 200 python scripts/layer_profile.py --batch 32 > $T/layers_dbl_n_bs32.txt 2>&1 || { tail $T/layers_dbl_n_bs32.txt; exit 1; }
head -2 $T/layers_dbl_n_bs16.txt
