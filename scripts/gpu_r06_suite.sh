#!/bin/bash
# Round 6: the whole GPU suite and smoke (as the driver runs them at round end).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_suite; mkdir -p $T
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $T/pytest_gpu.txt 2>&1 \
    || { grep -E "FAILED|Error" $T/pytest_gpu.txt | head -20; tail -40 $T/pytest_gpu.txt; exit 1; }
tail -2 $T/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 1; }
tail -3 $T/smoke.txt
