# Round 5: predict()'s two-slot in-place path: parity (ops + model predict tests), timing vs the session bench,
# host probe.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05as; mkdir -p $T
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_plugin.py -k "stem or input or predict or session or sharded or batch_max or forward or plugin" -x -q --timeout 120 --timeout-method thread > $T/parity.log 2>&1 || { tail -40 $T/parity.log; exit 1; }
tail -1 $T/parity.log
timeout -k 10 200 python scripts/predict_probe.py 2>&1 | grep -v amdgpu.ids | tee $T/probe.txt || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $T/bench_r$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --via-predict > $T/predict_r$r.json 2>/dev/null || exit 1
done
for f in $T/bench_r1.json $T/predict_r1.json $T/bench_r2.json $T/predict_r2.json; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $f
done
