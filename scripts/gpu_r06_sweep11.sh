#!/bin/bash
# Round 6: 4x8 lean DSConv tiles for 128 channels on the smallest grids (YDBL_LEAN_T48=1: config 3's bs4 sub-batch,
# 100 8x8 tiles on 256 CUs), parity (bit-identical to the chunked kernel) + same-process A/B, two sessions each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep11; mkdir -p $T
set -o pipefail
YDBL_LEAN_T48=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread \
    -k "dsconv_lean or dsconv_fused or dsc3k" > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
V=("base:" "t48:YDBL_LEAN_T48=1" "base2:" "t48b:YDBL_LEAN_T48=1")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 5 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -4
YDBL_LEAN_T48=1 timeout -k 10 240 python -u scripts/layer_profile.py --model s --batch 4 > $T/layers_s4_t48.txt 2>&1 || exit 1
grep -E "DSConv.k[37]s1 +128x40" $T/layers_s4_t48.txt | head -4
