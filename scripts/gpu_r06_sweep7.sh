#!/bin/bash
# Round 6: the new conv route defaults (N-blocked halo tiles for the VGPR-weight shapes and instead of 16-row tiles) vs
# the previous routes (YDBL_VW=1; YDBL_HALO_T16=1) on configs 2, 3 and 4, same process, interleaved; conv parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep7; mkdir -p $T
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread \
    -k "halo or vw or conv_dense or split_k or bottleneck" > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
V=("new:" "old:YDBL_VW=1;YDBL_HALO_T16=1")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 6 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -2
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 6 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -2
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 64 --rounds 3 --steps 10 > $T/s64.txt 2>&1 || exit 1
grep -v amdgpu $T/s64.txt | tail -2
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model l --batch 8 --imgsz 1280 --rounds 3 --steps 6 > $T/l8.txt 2>&1 || exit 1
grep -v amdgpu $T/l8.txt | tail -2
