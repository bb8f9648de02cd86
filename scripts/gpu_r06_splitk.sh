#!/bin/bash
# Round 6: split-K conv parity and A/B (config 3 per-rank DBL-s bs8, config 2 DBL-n bs32) + bs4 layer profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_splitk; mkdir -p $T
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
    -k "conv_dense or split_k or conv1x1 or halo or vw" > $T/pytest_conv.txt 2>&1 || { tail -30 $T/pytest_conv.txt; exit 1; }
timeout -k 10 300 python -u scripts/ab_bench.py "split:" "nosplit:YDBL_SPLITK=0" --model s --batch 8 --rounds 5 \
    --steps 60 > $T/ab_s8.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_bench.py "split:" "nosplit:YDBL_SPLITK=0" --model n --batch 32 --rounds 5 \
    --steps 40 > $T/ab_n32.txt 2>&1 || exit 1
timeout -k 10 240 python -u scripts/layer_profile.py --model s --batch 4 > $T/layers_s4.txt 2>&1
