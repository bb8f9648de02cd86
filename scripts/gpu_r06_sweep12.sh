#!/bin/bash
# Round 6: 8x16 lean DSConv tiles for 128 channels on small grids (YDBL_LEAN_T816=1: half the workgroups,
# 100 8x8 tiles on 256 CUs), parity (bit-identical to the chunked kernel) + same-process A/B, two sessions each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep12; mkdir -p $T
set -o pipefail
YDBL_LEAN_T816=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread \
    -k "dsconv_lean or dsconv_fused or dsc3k" > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
V=("base:" "t816:YDBL_LEAN_T816=1" "base2:" "t816b:YDBL_LEAN_T816=1")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 5 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -4
YDBL_LEAN_T816=1 timeout -k 10 240 python -u scripts/layer_profile.py --model s --batch 4 > $T/layers_s4_t816.txt 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 5 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -4
grep -E "DSConv.k[37]s1 +128x40" $T/layers_s4_t816.txt | head -4
