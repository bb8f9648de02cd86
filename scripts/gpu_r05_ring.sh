# Round 5: the LDS-DMA ring 3x3 kernel (YDBL_HALO_RING=TH[,WAVES]): parity, kbench of the halo shapes per variant
# (two rounds), then the bench workload A/B in one process.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05rg; mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "ring" > $T/pytest_ring.log 2>&1 || { tail -30 $T/pytest_ring.log; exit 1; }
tail -1 $T/pytest_ring.log
for r in 1 2; do
  for e in "-" "YDBL_HALO_RING=8" "YDBL_HALO_RING=16" "YDBL_HALO_RING=20" "YDBL_HALO_RING=16,8" "YDBL_HALO_RING=20,8"; do
    echo "== round $r env $e" >> $T/kbench.txt
    if [ "$e" = "-" ]; then timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/kbench.txt 2>&1 || exit 1
    else env $e timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/kbench.txt 2>&1 || exit 1; fi
  done
done
grep -v amdgpu.ids $T/kbench.txt | grep -v dsconv
timeout -k 10 400 python scripts/ab_bench.py "A:" "R16:YDBL_HALO_RING=16" "R20:YDBL_HALO_RING=20" "R16w8:YDBL_HALO_RING=16,8" \
  --rounds 4 > $T/ab_bench.txt 2>&1 || { tail -5 $T/ab_bench.txt; exit 1; }
tail -6 $T/ab_bench.txt
timeout -k 10 1000 python -u scripts/fp8_calibrate.py > $T/fp8_calibrate_fwd.txt 2>&1; rc=$?; tail -10 $T/fp8_calibrate_fwd.txt
cp tests/golden/fp8_calib_yolov13s_DBL_nc3.json $T/fp8_calib_fwd.json 2>/dev/null; exit $rc
