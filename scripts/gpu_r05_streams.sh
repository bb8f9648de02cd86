# Round 5: sub-batch graph count A/B with the one-graph branch runner (DBL-n bs32, DBL-s bs64), same process.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05st3; mkdir -p $T
set -o pipefail
timeout -k 10 300 python scripts/ab_bench.py "S2:" "S3:STREAMS=3" "S4:STREAMS=4" --rounds 4 2>&1 | grep -v amdgpu.ids | tee $T/n.txt || exit 1
timeout -k 10 400 python scripts/ab_bench.py "S2:" "S3:STREAMS=3" "S4:STREAMS=4" --model s --batch 64 --rounds 3 --steps 20 2>&1 | grep -v amdgpu.ids | tee $T/s.txt || exit 1
