#!/bin/bash
# Round 6: this round's routing defaults (cur) vs round 5's (prev: one-image halo workgroups, DSC3k 1x1 fusions, LSK
# fused at every dim, fused DWConv -> Conv1x1 at every width, VGPR-weight 3x3s, 16-row halo tiles), each as TWO
# sessions (cur/cur2, prev/prev2) so the session-to-session bias shows, same process, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_defaults; mkdir -p $T
set -o pipefail
P="YDBL_HALO_NB=1;YDBL_CV1_FUSE=1;YDBL_CV3_FUSE=1;YDBL_LSK_FUSE=1;YDBL_DWPW=1;YDBL_VW=1;YDBL_HALO_T16=1"
V=("cur:" "prev:$P" "cur2:" "prev2:$P")
timeout -k 10 900 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 6 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -4
timeout -k 10 900 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 6 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -4
timeout -k 10 900 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 64 --rounds 3 --steps 10 > $T/s64.txt 2>&1 || exit 1
grep -v amdgpu $T/s64.txt | tail -4
