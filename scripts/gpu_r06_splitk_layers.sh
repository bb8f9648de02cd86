#!/bin/bash
# Round 6: in-graph layer profiles with split-K on / off (YDBL_SPLITK), DBL-l 1280 bs4 and DBL-s 640 bs4 sub-batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sklayers; mkdir -p $T
set -o pipefail
for m in "l 1280" "s 640"; do
  set -- $m
  timeout -k 10 300 python -u scripts/layer_profile.py --model $1 --batch 4 --imgsz $2 > $T/layers_$1_on.txt 2>&1 || exit 1
  YDBL_SPLITK=0 timeout -k 10 300 python -u scripts/layer_profile.py --model $1 --batch 4 --imgsz $2 > $T/layers_$1_off.txt 2>&1 || exit 1
done
