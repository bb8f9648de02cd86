cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/br
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/br/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/br/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/br/b$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])" gpurun_out/br/b$r.json
done
for a in "--model s --batch 64" "--model l --batch 8 --imgsz 1280 --steps 20 --warmup 5" "--model s --fp8"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline $a 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'])" || exit 1
done
timeout -k 10 300 python scripts/graph_branch_probe.py
