#!/bin/bash
# Round 6: every plan-builder fusion switched off in turn, same process, interleaved rounds (scripts/ab_bench.py),
# DBL-n bs32 (config 2) and DBL-s bs8 (config 3 per rank): does each fusion still pay in the final two-branch layout?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; T=gpurun_out/r06_sweep; mkdir -p $T
set -o pipefail
V=("base:" "nocv1:YDBL_NO_CV1_FUSE=1" "nocv3:YDBL_NO_CV3_FUSE=1" "nomerge:YDBL_NO_MERGE=1" "nopad:YDBL_NO_FUSE_PAD=1"
   "lskunf:YDBL_LSK_UNFUSED=1" "ds2off:YDBL_DS2_OFF=1" "nobneck:YDBL_NO_BNECK=1")
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model n --batch 32 --rounds 4 --steps 30 > $T/sweep_n32.txt 2>&1 || { tail -20 $T/sweep_n32.txt; exit 1; }
grep -v amdgpu $T/sweep_n32.txt | tail -8
timeout -k 10 600 python -u scripts/ab_bench.py "${V[@]}" --model s --batch 8 --rounds 4 --steps 40 > $T/sweep_s8.txt 2>&1 || { tail -20 $T/sweep_s8.txt; exit 1; }
grep -v amdgpu $T/sweep_s8.txt | tail -8
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "halo_nblock or stem2" \
    > $T/pytest_nb.txt 2>&1 || { tail -30 $T/pytest_nb.txt; exit 1; }
tail -1 $T/pytest_nb.txt
timeout -k 10 400 python -u scripts/ab_bench.py "nb1:" "nb2:YDBL_HALO_NB=2" --model n --batch 32 --rounds 5 > $T/ab_nb_n32.txt 2>&1 || exit 1
grep -v amdgpu $T/ab_nb_n32.txt | tail -2
timeout -k 10 400 python -u scripts/ab_bench.py "nb1:" "nb2:YDBL_HALO_NB=2" --model s --batch 8 --rounds 5 --steps 60 > $T/ab_nb_s8.txt 2>&1 || exit 1
grep -v amdgpu $T/ab_nb_s8.txt | tail -2
YDBL_HALO_NB=2 timeout -k 10 240 python -u scripts/layer_profile.py --model n --batch 16 > $T/layers_n16_nb2.txt 2>&1 || exit 1
grep -E "Conv3x3 .*k3 s1" $T/layers_n16_nb2.txt
