#!/bin/bash
# Round 6: the remaining routing switches in the final layout (N-blocking variants, lean vs chunked DSConv, hypergraph,
# stem pair, split-K), same process, interleaved rounds, DBL-n bs32 and DBL-s bs8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep3; mkdir -p $T
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "halo_nblock" \
    > $T/pytest_nb.txt 2>&1 || { tail -30 $T/pytest_nb.txt; exit 1; }
V=("base:" "nb4:YDBL_HALO_NB=4" "nb2w:YDBL_HALO_NB=2w" "nolean:YDBL_DS_LEAN=0" "hgunf:YDBL_HG_UNFUSED=1"
   "nostem2:YDBL_NO_STEM2=1" "nosplitk:YDBL_SPLITK=0")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 4 --steps 30 > $T/n32.txt 2>&1 || { tail -20 $T/n32.txt; exit 1; }
grep -v amdgpu $T/n32.txt | tail -8
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 4 --steps 40 > $T/s8.txt 2>&1 || { tail -20 $T/s8.txt; exit 1; }
grep -v amdgpu $T/s8.txt | tail -8
