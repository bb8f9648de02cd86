#!/bin/bash
# Round 6: sub-batch graphs on CU-partitioned streams (scripts/cu_mask_probe.py) for configs 2 and 3; the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_cumask; mkdir -p $T
set -o pipefail
timeout -k 10 300 python -u scripts/cu_mask_probe.py --model n --batch 32 > $T/cumask_n32.txt 2>&1 || { tail -20 $T/cumask_n32.txt; exit 1; }
grep -v amdgpu $T/cumask_n32.txt
timeout -k 10 300 python -u scripts/cu_mask_probe.py --model s --batch 8 > $T/cumask_s8.txt 2>&1 || { tail -20 $T/cumask_s8.txt; exit 1; }
grep -v amdgpu $T/cumask_s8.txt
timeout -k 10 300 python bench.py > $T/bench.log 2>&1 || { tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-600
