#!/bin/bash
# full GPU suite + smoke, then the round-3 records (scripts/gpu_r03_final.sh) on the final code
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=gpurun_out/${1:-r03fin2}; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $T/pytest_gpu.log 2>&1; rc=$?
tail -2 $T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 3; }
tail -2 $T/smoke.log
bash scripts/gpu_r03_final.sh ${1:-r03fin2}
