# Round 5: the whole GPU suite + smoke (as the driver runs them at round end).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05full; mkdir -p $T
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $T/pytest_gpu.log 2>&1; rc=$?
tail -5 $T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 1; }
tail -3 $T/smoke.log
