#!/bin/bash
# Round 6: targeted GPU tests + bench lines of configs 2 (session, predict), 3, 4 (no rocprof).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_quick; mkdir -p $T
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_plugin.py -q \
    --timeout 300 --timeout-method thread -k "split_k or conv_dense or predict or plugin or nms" > $T/pytest.txt 2>&1 \
    || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
for cfg in "c2:--model n" "c2p:--model n --via-predict" "c3:--model s --batch 8" "c4:--model l --batch 8 --imgsz 1280 --steps 20 --warmup 5"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-roofline > $T/$n.log 2>&1 || { echo "bench $n failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $T/$n.log $n
done
timeout -k 10 400 python -u scripts/val_timing.py > $T/val_timing.txt 2>&1 || { tail -20 $T/val_timing.txt; exit 1; }
tail -6 $T/val_timing.txt
