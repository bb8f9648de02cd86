# Round 5 call 7: XCD-aware tile order A/B (scripts/gpu_r05_xcd.sh), then the DSC3k chain experiment: parity
# (bit-identical to the four launches), in-graph cost against the unchained launches, per-stage barrier stamps.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05c7; mkdir -p $T
set -o pipefail
bash scripts/gpu_r05_xcd.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "dsc3k_chain or dsconv_lean" -x -q --timeout 120 --timeout-method thread > $T/chain_parity.log 2>&1 || { tail -30 $T/chain_parity.log; exit 1; }
tail -2 $T/chain_parity.log
for r in 1 2; do
  for m in 0 1 2; do
    YDBL_DSC3K_CHAIN=$m timeout -k 10 120 python scripts/kbench.py "dsc3k" 2>&1 | grep "us/launch" | sed "s/^/mode $m r$r: /" >> $T/chain_kbench.txt || exit 1
  done
done
cat $T/chain_kbench.txt
for m in 1 2; do
  YDBL_DSC3K_CHAIN=$m timeout -k 10 120 python scripts/chain_stamps.py 16 20 >> $T/chain_stamps.txt 2>&1 || { tail -20 $T/chain_stamps.txt; exit 1; }
done
cat $T/chain_stamps.txt
timeout -k 10 500 python scripts/ab_bench.py "A:" "CHAIN1:YDBL_DSC3K_CHAIN=1" "CHAIN2:YDBL_DSC3K_CHAIN=2" --rounds 4 > $T/chain_ab.txt 2>&1 || { tail -20 $T/chain_ab.txt; exit 1; }
tail -8 $T/chain_ab.txt
