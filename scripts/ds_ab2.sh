cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03f; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dsconv or detect or dsc3k or blocks or stem" > gpurun_out/r03f/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03f/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/kbench.py pair dsconv 2>&1 | grep us/launch
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03f/bench.log 2>&1; tail -1 gpurun_out/r03f/bench.log | cut -c1-300
