cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03h; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "split_k or conv_dense or conv1x1" > gpurun_out/r03h/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03h/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== split"; timeout -k 10 120 python scripts/kbench.py "conv " 2>&1 | grep us/launch
echo "== nosplit"; YDBL_NO_SPLITK=1 timeout -k 10 120 python scripts/kbench.py "conv " 2>&1 | grep us/launch
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03h/bench.log 2>&1; tail -1 gpurun_out/r03h/bench.log | cut -c1-200
