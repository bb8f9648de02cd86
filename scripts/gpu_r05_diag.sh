# Round 5: where the halo 3x3 kernel's time goes (timing-only YDBL_HALO_DIAG builds: 1 no weight restage, 2 no halo
# restage, 4 no MFMAs; combinations), kbench bs16 head shapes, two rounds; plus the fp8 greedy calibration.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05dg; mkdir -p $T
for r in 1 2; do for d in 0 1 2 3 4 5 6 7; do
  echo "== round $r diag $d" >> $T/kbench.txt
  YDBL_HALO_DIAG=$d timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "256->32 k3s1@80 bs16" >> $T/kbench.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $T/kbench.txt | grep -v dsconv
timeout -k 10 900 python -u scripts/fp8_calibrate.py > $T/fp8_calibrate_greedy.txt 2>&1; rc=$?; tail -12 $T/fp8_calibrate_greedy.txt
cp tests/golden/fp8_calib_yolov13s_DBL_nc3.json $T/fp8_calib_greedy.json 2>/dev/null; exit $rc
