# Round 5: the benched layouts against the oracle (e2e + sharded nccl + predict layout), then the default bench and
# the public-API bench.  usage: bash scripts/gpu_r05_parity.sh TAG
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=${1:-r05p}; mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_model.py -m gpu -v -s --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/$T/pytest_e2e_model.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/$T/pytest_e2e_model.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2>gpurun_out/$T/bench.err || exit 1
cut -c1-300 gpurun_out/$T/bench.json
timeout -k 10 300 python bench.py --via-predict > gpurun_out/$T/bench_predict.json 2>gpurun_out/$T/bench_predict.err || exit 1
cut -c1-300 gpurun_out/$T/bench_predict.json
