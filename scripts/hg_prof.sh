cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03k; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "hypergraph or hyperace or c3ah" > gpurun_out/r03k/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03k/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/kbench.py "hg " 2>&1 | grep us/launch
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r03k/prof -o hg -- python scripts/kbench.py "hg " --eager=20 > gpurun_out/r03k/prof.log 2>&1
