#!/bin/bash
# Round 6: combinations from the fusion-switch sweep (r06_fusion_switch_sweep.txt) on configs 2, 3 (per rank and
# one-GPU bs64) and 4, same process, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep2; mkdir -p $T
set -o pipefail
timeout -k 10 500 python -u scripts/ab_bench.py "base:" "nb2:YDBL_HALO_NB=2" "c13:YDBL_NO_CV1_FUSE=1;YDBL_NO_CV3_FUSE=1" \
    "c13nb2:YDBL_NO_CV1_FUSE=1;YDBL_NO_CV3_FUSE=1;YDBL_HALO_NB=2" --model n --batch 32 --rounds 5 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -4
timeout -k 10 500 python -u scripts/ab_bench.py "base:" "lsk:YDBL_LSK_UNFUSED=1" "lskc1:YDBL_LSK_UNFUSED=1;YDBL_NO_CV1_FUSE=1" \
    "lskc13nb2:YDBL_LSK_UNFUSED=1;YDBL_NO_CV1_FUSE=1;YDBL_NO_CV3_FUSE=1;YDBL_HALO_NB=2" --model s --batch 8 --rounds 5 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -4
timeout -k 10 500 python -u scripts/ab_bench.py "base:" "lsk:YDBL_LSK_UNFUSED=1" "c13nb2:YDBL_NO_CV1_FUSE=1;YDBL_NO_CV3_FUSE=1;YDBL_HALO_NB=2" \
    --model s --batch 64 --rounds 3 --steps 10 > $T/s64.txt 2>&1 || exit 1
grep -v amdgpu $T/s64.txt | tail -3
timeout -k 10 500 python -u scripts/ab_bench.py "base:" "nb2:YDBL_HALO_NB=2" "lsk:YDBL_LSK_UNFUSED=1" --model l --batch 8 --imgsz 1280 \
    --rounds 3 --steps 6 > $T/l8.txt 2>&1 || exit 1
grep -v amdgpu $T/l8.txt | tail -3
