cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2>gpurun_out/final/bench.err || exit 1; cut -c1-200 gpurun_out/final/bench.json
python -c "import json; d=json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(r['frac'], r['traffic'], r['mfma_busy'], r['pmc_summary'], r['network']['frac'])"
