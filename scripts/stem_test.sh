cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03m; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "stem or e2e_n640 or smoke" > gpurun_out/r03m/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03m/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/kbench.py stem2 "conv 16" "conv 32" "bneck"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03m/bench.log 2>&1; tail -1 gpurun_out/r03m/bench.log | cut -c1-180
