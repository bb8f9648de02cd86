# Round 5: per-stage stamps of the DSC3k chain experiment (agent-scope and XCD-local group barriers).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05st; mkdir -p $T
set -o pipefail
for m in 1 2; do
  YDBL_DSC3K_CHAIN=$m timeout -k 10 120 python scripts/chain_stamps.py 16 20 >> $T/chain_stamps.txt 2>&1 || { tail -20 $T/chain_stamps.txt; exit 1; }
done
grep -v amdgpu.ids $T/chain_stamps.txt
