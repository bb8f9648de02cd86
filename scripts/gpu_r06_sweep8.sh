#!/bin/bash
# Round 6: the two conv route defaults one at a time on the headline config (DBL-n bs32), 8 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep8; mkdir -p $T
set -o pipefail
V=("new:" "vw1:YDBL_VW=1" "t16:YDBL_HALO_T16=1" "old:YDBL_VW=1;YDBL_HALO_T16=1")
timeout -k 10 900 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 8 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -4
