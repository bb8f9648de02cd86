# Round 5: halo kernel k-steps per chunk (YDBL_HALO_KS) / tile height / channel slice: parity under KS=2, kbench of
# the halo shapes per variant (two rounds), then the bench workload A/B in one process (scripts/ab_bench.py).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05ks; mkdir -p $T
YDBL_HALO_KS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "halo or fp8" > $T/pytest_ks2.log 2>&1 || { tail -20 $T/pytest_ks2.log; exit 1; }
tail -1 $T/pytest_ks2.log
for r in 1 2; do
  for e in "-" "YDBL_HALO_KS=2" "YDBL_HALO_TH=4" "YDBL_HALO_TH=4 YDBL_HALO_KS=2" "YDBL_HALO_TH=8 YDBL_HALO_NTN=1" "YDBL_HALO_TH=8 YDBL_HALO_NTN=1 YDBL_HALO_KS=2"; do
    echo "== round $r env $e" >> $T/kbench.txt
    if [ "$e" = "-" ]; then timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/kbench.txt 2>&1 || exit 1
    else env $e timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/kbench.txt 2>&1 || exit 1; fi
  done
done
grep -v amdgpu.ids $T/kbench.txt | grep -v dsconv
timeout -k 10 400 python scripts/ab_bench.py "A:" "KS2:YDBL_HALO_KS=2" "TH4:YDBL_HALO_TH=4" "TH4KS2:YDBL_HALO_TH=4,YDBL_HALO_KS=2" \
  --rounds 4 > $T/ab_bench.txt 2>&1 || { tail -5 $T/ab_bench.txt; exit 1; }
tail -8 $T/ab_bench.txt
