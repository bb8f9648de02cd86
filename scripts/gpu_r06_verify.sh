#!/bin/bash
# Round 6 (re-entry): verify on hardware -- NMS radix select above 8192 candidates, the halo tile for unsplittable
# small-map 3x3s, split-K on the larger maps (YDBL_SPLITK_BIG), the one-launch DSBottleneck (YDBL_DSB_PAIR): parity,
# same-process A/Bs on configs 2 and 3, in-graph layer profiles, NMS timing, val() timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_verify; mkdir -p $T
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread \
    -k "dsb_pair or dsc3k or dsconv_lean or nms or conv_dense or split_k or halo or vw" > $T/pytest_ops.txt 2>&1 \
    || { tail -30 $T/pytest_ops.txt; exit 1; }
tail -1 $T/pytest_ops.txt
timeout -k 10 400 python -u scripts/ab_bench.py "new:" "nopair:YDBL_DSB_PAIR=0" "nobig:YDBL_SPLITK_BIG=0" --model n \
    --batch 32 --rounds 5 > $T/ab_n32.txt 2>&1 || exit 1
grep -v amdgpu $T/ab_n32.txt | tail -4
timeout -k 10 240 python -u scripts/layer_profile.py --model n --batch 16 > $T/layers_n16.txt 2>&1 || exit 1
head -16 $T/layers_n16.txt
timeout -k 10 300 python -u scripts/ab_bench.py "halo:" "wsk:YDBL_HALO_SMALL=0" "nopair:YDBL_DSB_PAIR=0" --model s \
    --batch 8 --rounds 5 --steps 60 > $T/ab_s8.txt 2>&1 || exit 1
grep -v amdgpu $T/ab_s8.txt | tail -4
timeout -k 10 240 python -u scripts/layer_profile.py --model s --batch 4 > $T/layers_s4.txt 2>&1 || exit 1
head -3 $T/layers_s4.txt
timeout -k 10 300 python -u scripts/nms_wide_bench.py > $T/nms_wide_bench.txt 2>&1 || { tail -20 $T/nms_wide_bench.txt; exit 1; }
grep -v amdgpu $T/nms_wide_bench.txt | tail -14
timeout -k 10 400 python -u scripts/val_timing.py > $T/val_timing.txt 2>&1 || { tail -20 $T/val_timing.txt; exit 1; }
tail -6 $T/val_timing.txt
