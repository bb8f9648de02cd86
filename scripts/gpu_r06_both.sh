#!/bin/bash
# Round 6: NMS (tests, timing, stamps) then split-K conv (tests, A/B, bs4 layer profile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
set -o pipefail
bash scripts/gpu_r06_nms.sh || { echo "nms failed"; tail -30 gpurun_out/r06_nms/pytest_nms.txt gpurun_out/r06_nms/pytest_model.txt; exit 1; }
bash scripts/gpu_r06_splitk.sh || { echo "splitk failed"; exit 1; }
