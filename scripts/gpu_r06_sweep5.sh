#!/bin/bash
# Round 6: confirmation A/Bs of the two Detect-head switches that measured above noise in r06_sweep4 (the class conv
# riding on the second DWConv -> Conv1x1 pair on DBL-n; the fused DWConv -> Conv1x1 pairs on DBL-s), more rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep5; mkdir -p $T
set -o pipefail
timeout -k 10 600 python -u scripts/ab_bench.py "base:" "notail:YDBL_NO_CLS_TAIL=1" --model n --batch 32 --rounds 8 --steps 40 > $T/n32.txt 2>&1 || exit 1
grep -v amdgpu $T/n32.txt | tail -2
timeout -k 10 600 python -u scripts/ab_bench.py "base:" "nodwpw:YDBL_NO_DWPW=1" --model s --batch 8 --rounds 8 --steps 40 > $T/s8.txt 2>&1 || exit 1
grep -v amdgpu $T/s8.txt | tail -2
timeout -k 10 600 python -u scripts/ab_bench.py "base:" "nodwpw:YDBL_NO_DWPW=1" --model s --batch 64 --rounds 4 --steps 10 > $T/s64.txt 2>&1 || exit 1
grep -v amdgpu $T/s64.txt | tail -2
timeout -k 10 600 python -u scripts/ab_bench.py "base:" "nodwpw:YDBL_NO_DWPW=1" --model l --batch 8 --imgsz 1280 --rounds 3 --steps 6 > $T/l8.txt 2>&1 || exit 1
grep -v amdgpu $T/l8.txt | tail -2
