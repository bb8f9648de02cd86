# Round 5 call 3: plugin / predict / fp8-calibration tests, the fp8 calibration record + config-5 sweep, the
# via-predict bench, the memory-path probe of the halo convs.  A failed test does not stop the later steps; a
# crash, abort or time-out does.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05i3; mkdir -p $T
step() { local rc=$1; shift; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP: $* rc=$rc"; exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_model.py -m gpu -v -s --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "plugin or forward or predict or fp8_calibration" > $T/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $T/pytest.log | tail -3; step $rc pytest
timeout -k 10 600 python -u scripts/fp8_calibrate.py > $T/fp8_calibrate.txt 2>&1; rc=$?; tail -8 $T/fp8_calibrate.txt; step $rc fp8
cp tests/golden/fp8_calib_yolov13s_DBL_nc3.json $T/ 2>/dev/null
timeout -k 10 300 python bench.py --via-predict > $T/bench_predict.json 2>$T/bench_predict.err; rc=$?; cut -c1-200 $T/bench_predict.json; step $rc bench
bash scripts/gpu_r05_memprobe.sh r05mem
