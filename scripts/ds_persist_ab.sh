cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03e; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dsconv or detect or dsc3k or blocks" > gpurun_out/r03e/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03e/pytest.log; [ $rc -eq 0 ] || exit $rc
for pc in 0 2 3; do echo "== persist $pc"; YDBL_DS_PERSIST=$pc timeout -k 10 120 python scripts/kbench.py pair dsconv 2>&1 | grep us/launch; done
echo "== chunked"; YDBL_DS_LEAN=0 timeout -k 10 120 python scripts/kbench.py pair dsconv 2>&1 | grep us/launch
