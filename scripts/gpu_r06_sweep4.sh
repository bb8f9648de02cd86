#!/bin/bash
# Round 6: the Detect-head fusions switched off in turn (box branch as one bottleneck launch, the 64->64 3x3 pair,
# DWConv -> Conv1x1 pairs, the class conv riding on the second pair), same process, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep4; mkdir -p $T
set -o pipefail
V=("base:" "nobox3:YDBL_NO_BOX3=1" "nopair3:YDBL_NO_PAIR3=1" "nodwpw:YDBL_NO_DWPW=1" "notail:YDBL_NO_CLS_TAIL=1")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 5 --steps 30 > $T/n32.txt 2>&1 || { tail -20 $T/n32.txt; exit 1; }
grep -v amdgpu $T/n32.txt | tail -5
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 5 --steps 40 > $T/s8.txt 2>&1 || { tail -20 $T/s8.txt; exit 1; }
grep -v amdgpu $T/s8.txt | tail -5
