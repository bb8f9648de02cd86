#!/bin/bash
# Round 6: the block-GEMM workgroup target (YDBL_IGEMM_WANT scales it by v / 512: 128 / 256 = bigger tiles, fewer
# workgroups, less weight restaging; 1024 = more), same process, interleaved rounds; then the PMC families of the final
# code on the roofline's single-stream workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep9; mkdir -p $T
set -o pipefail
V=("base:" "w128:YDBL_IGEMM_WANT=128" "w256:YDBL_IGEMM_WANT=256" "w1024:YDBL_IGEMM_WANT=1024" "base2:")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 5 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -5
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 5 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -5
