#!/bin/bash
# Round 6: sub-batch graphs per step re-measured with the final routing (same process, interleaved): DBL-s bs64 (config
# 3 on one GPU) 2 / 4 graphs, DBL-n bs32 2 / 4, DBL-l 1280 bs8 1 / 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_streams; mkdir -p $T
set -o pipefail
timeout -k 10 500 python -u scripts/ab_bench.py "S2:" "S4:STREAMS=4" --model s --batch 64 --rounds 4 --steps 10 > $T/s64.txt 2>&1 || exit 1
grep -v amdgpu $T/s64.txt | tail -2
timeout -k 10 500 python -u scripts/ab_bench.py "S2:" "S4:STREAMS=4" --model n --batch 32 --rounds 5 --steps 30 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -2
timeout -k 10 500 python -u scripts/ab_bench.py "S2:" "S1:STREAMS=1" --model l --batch 8 --imgsz 1280 --rounds 3 --steps 6 > $T/l8.txt 2>&1 || exit 1
grep -v amdgpu $T/l8.txt | tail -2
