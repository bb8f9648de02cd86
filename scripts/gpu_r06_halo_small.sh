#!/bin/bash
# Round 6: the halo tile for unsplittable small-map 3x3s with Cout >= 128 (YDBL_HALO_SMALL): parity, same-process
# A/B on config 3's per-rank workload and config 4, the bs4 layer profile (split-K fixed), val() timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_halo_small; mkdir -p $T
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
    -k "conv_dense or split_k or halo or vw" > $T/pytest_conv.txt 2>&1 || { tail -30 $T/pytest_conv.txt; exit 1; }
tail -1 $T/pytest_conv.txt
timeout -k 10 300 python -u scripts/ab_bench.py "halo:" "wsk:YDBL_HALO_SMALL=0" --model s --batch 8 --rounds 5 \
    --steps 60 > $T/ab_s8.txt 2>&1 || exit 1
grep -v amdgpu $T/ab_s8.txt | tail -3
timeout -k 10 400 python -u scripts/ab_bench.py "halo:" "wsk:YDBL_HALO_SMALL=0" --model l --batch 8 --imgsz 1280 \
    --rounds 3 --steps 10 > $T/ab_l8.txt 2>&1 || exit 1
grep -v amdgpu $T/ab_l8.txt | tail -3
timeout -k 10 240 python -u scripts/layer_profile.py --model s --batch 4 > $T/layers_s4.txt 2>&1 || exit 1
head -3 $T/layers_s4.txt
timeout -k 10 400 python -u scripts/val_timing.py > $T/val_timing.txt 2>&1 || { tail -20 $T/val_timing.txt; exit 1; }
tail -6 $T/val_timing.txt
