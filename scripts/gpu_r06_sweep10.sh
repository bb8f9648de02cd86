#!/bin/bash
# Round 6: 16-row Bottleneck tiles for every c_mid < 64 launch (YDBL_BNECK_T16=1: DBL-n's four c64 Bottlenecks at 80^2
# take 16-row tiles instead of 8/9-row ones -- less halo recompute, half the workgroups), parity + same-process A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep10; mkdir -p $T
set -o pipefail
YDBL_BNECK_T16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "bottleneck" \
    > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
V=("base:" "t16:YDBL_BNECK_T16=1" "base2:" "t16b:YDBL_BNECK_T16=1")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 5 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -4
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 5 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -4
