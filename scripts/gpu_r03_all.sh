#!/bin/bash
# streams A/B, then the round-3 records (configs 2-5 + rocprof, single-stream summary, PMC families), and the
# config-5 mAP drops with their printout
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=gpurun_out/${1:-r03rec}; mkdir -p $T
bash scripts/streams_ab.sh > $T/streams_ab.txt 2>&1; cat $T/streams_ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "map50_config5 or fp8_config5" > $T/fp8_tests.log 2>&1; rc=$?
grep -E "mAP50|s640 bs32 fp8|passed|failed" $T/fp8_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r03_records.sh ${1:-r03rec}
