# DSC3k chain: bit-identity test, in-graph layer profile and bench A/B (YDBL_DSC3K_CHAIN=1 / 0)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/chain
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "chain" > gpurun_out/chain/test.log 2>&1; rc=$?; tail -3 gpurun_out/chain/test.log; [ $rc -eq 0 ] || exit $rc
for c in 1 0; do
  YDBL_DSC3K_CHAIN=$c timeout -k 10 200 python scripts/layer_profile.py --batch 16 > gpurun_out/chain/layers_bs16_chain$c.txt 2>&1 || exit 1
  head -3 gpurun_out/chain/layers_bs16_chain$c.txt | tail -2; grep -E "DSC3k|dsconv" gpurun_out/chain/layers_bs16_chain$c.txt | head -4
done
for r in 1 2; do for c in 1 0; do
  YDBL_DSC3K_CHAIN=$c timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/chain/bench_c${c}_r$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/chain/bench_c${c}_r$r.json
done; done
