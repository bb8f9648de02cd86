# Round 5 call: double-buffered ring variant A/B (kbench), the per-launch conv HBM fetch table (PMC), the fp8
# calibration with forward selection.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05c6; mkdir -p $T
for r in 1 2; do
  for e in "-" "YDBL_HALO_RING=8,4,2" "YDBL_HALO_RING=16,4,2"; do
    echo "== round $r env $e" >> $T/kbench.txt
    if [ "$e" = "-" ]; then timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/kbench.txt 2>&1 || exit 1
    else env $e timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/kbench.txt 2>&1 || exit 1; fi
  done
done
grep -v amdgpu.ids $T/kbench.txt | grep -v dsconv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $T/fetch -o run -- python scripts/pmc_conv_fetch.py run $T/conv_steps.json > $T/fetch.log 2>&1 || { tail -5 $T/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $T/write -o run -- python scripts/pmc_conv_fetch.py run $T/conv_steps.json > $T/write.log 2>&1 || { tail -5 $T/write.log; exit 1; }
python scripts/pmc_conv_fetch.py report $T/conv_steps.json $T/fetch $T/write > $T/conv_fetch_table.txt 2>&1; tail -40 $T/conv_fetch_table.txt
timeout -k 10 1000 python -u scripts/fp8_calibrate.py > $T/fp8_calibrate_fwd.txt 2>&1; rc=$?; tail -10 $T/fp8_calibrate_fwd.txt
cp tests/golden/fp8_calib_yolov13s_DBL_nc3.json $T/fp8_calib_fwd.json 2>/dev/null; exit $rc
