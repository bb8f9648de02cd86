# Round-4 GPU pass: the new / changed tests verbosely (-s: the |gpu - oracle fp32| reports), then the whole GPU
# suite, smoke and the default bench line.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "forward or nccl" > gpurun_out/r04/new_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r04/new_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_e2e.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04/e2e.log 2>&1; rc=$?; tail -3 gpurun_out/r04/e2e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_e2e.py > gpurun_out/r04/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r04/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
timeout -k 10 400 python bench.py > gpurun_out/r04/bench.json 2>gpurun_out/r04/bench.err || exit 1; cut -c1-300 gpurun_out/r04/bench.json
