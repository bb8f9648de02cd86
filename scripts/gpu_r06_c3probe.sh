#!/bin/bash
# Round 6: config-3 per-rank workload (DBL-s 640 bs8) -- stream layouts and in-graph layer profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=gpurun_out/r06_c3probe; mkdir -p $T; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 240 python -u scripts/ab_bench.py "S1:STREAMS=1" "S2:STREAMS=2" "S3:STREAMS=3" "S4:STREAMS=4" \
    --model s --batch 8 --rounds 5 --steps 60 > $T/streams_s8.txt 2>&1 &&
timeout -k 10 240 python -u scripts/layer_profile.py --model s --batch 8 > $T/layers_s8.txt 2>&1 &&
timeout -k 10 240 python -u scripts/layer_profile.py --model s --batch 4 > $T/layers_s4.txt 2>&1
