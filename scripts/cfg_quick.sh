cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r03n
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dsconv or dsc3k or blocks or detect" > gpurun_out/r03n/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03n/pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "--model n" "--model s --batch 64" "--model l --batch 8 --imgsz 1280 --steps 20 --warmup 5" "--model s"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline $a 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'])"
done
