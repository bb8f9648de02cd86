#!/bin/bash
# Round 6: conv routing decisions made on single-launch latency, re-measured in the two-branch layout: the VGPR-weight
# 3x3 routes (YDBL_VW=0 -> halo tile), 16-row halo tiles (YDBL_HALO_T16=0 -> 8-row, N-blocked), half-height
# wave-split-K tiles (YDBL_WSK_HALF=0), same process, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep6; mkdir -p $T
set -o pipefail
V=("base:" "novw:YDBL_VW=0" "not16:YDBL_HALO_T16=0" "nohalf:YDBL_WSK_HALF=0")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 6 --steps 30 > $T/n32.txt 2>&1 || { tail -20 $T/n32.txt; exit 1; }
grep -v amdgpu $T/n32.txt | tail -4
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 6 --steps 40 > $T/s8.txt 2>&1 || { tail -20 $T/s8.txt; exit 1; }
grep -v amdgpu $T/s8.txt | tail -4
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 64 --rounds 3 --steps 10 > $T/s64.txt 2>&1 || { tail -20 $T/s64.txt; exit 1; }
grep -v amdgpu $T/s64.txt | tail -4
