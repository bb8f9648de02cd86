#!/bin/bash
# Round 6 final records, part 1: the whole GPU suite + smoke, then BASELINE configs 2-3 (bench line + rocprofv3 summary).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
set -o pipefail
bash scripts/gpu_r06_suite.sh || exit 1
bash scripts/gpu_configs.sh r06cfg 1 || exit 1
