#!/bin/bash
# BASELINE configs 3-5 on one MI355X + PMC HBM traffic of the default bench (tag = $1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=gpurun_out/${1:-cfg}; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model s --batch 64 --no-cpu-baseline > $T/s_bs64.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model l --batch 8 --imgsz 1280 --steps 20 --warmup 5 --no-cpu-baseline > $T/l_1280_bs8.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model s --no-cpu-baseline > $T/s_bs32.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model s --fp8 --no-cpu-baseline > $T/s_bs32_fp8.log 2>&1 || exit 1
bash scripts/pmc.sh ${1:-cfg}/pmc > $T/pmc.log 2>&1 || exit 1
for f in $T/*.log; do echo "$f: $(tail -1 $f | cut -c1-200)"; done
