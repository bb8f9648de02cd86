#!/bin/bash
# Round 6 final records, part 2: BASELINE configs 4-5, PMC families of the bench workload (hash-matched traffic for the
# bench line), bench vs rocprofv3 per-launch check, in-graph layer profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_final2; mkdir -p $T
set -o pipefail
bash scripts/gpu_configs.sh r06cfg 2 || exit 1
bash scripts/pmc_families.sh r06pmc profiles/r06/r06_pmc_families.json --model n || exit 1
bash scripts/roofline_check.sh r06rfchk > $T/rfchk.txt 2>&1 || { tail -20 $T/rfchk.txt; exit 1; }
tail -12 $T/rfchk.txt
for c in "n 32" "n 16" "s 4" "s 8"; do
  set -- $c
  timeout -k 10 240 python -u scripts/layer_profile.py --model $1 --batch $2 > $T/layers_$1_bs$2.txt 2>&1 || exit 1
  head -2 $T/layers_$1_bs$2.txt | tail -1
done
