# Bottleneck 10-row tiles (YDBL_BNECK_TH=10 for every auto-tiled launch): parity, kbench, layer profile, bench A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/bth
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "bottleneck or detect_box" > gpurun_out/bth/test.log 2>&1; rc=$?; tail -1 gpurun_out/bth/test.log; [ $rc -eq 0 ] || exit $rc
for th in 0 10; do
  YDBL_BNECK_TH=$th timeout -k 10 300 python scripts/kbench.py bneck box3 > gpurun_out/bth/kb_th$th.txt 2>&1 || exit 1
done
paste gpurun_out/bth/kb_th0.txt gpurun_out/bth/kb_th10.txt | awk -F'\t' '{printf "%-44s %8s %8s\n", substr($1,1,42), substr($1,42,9), substr($2,42,9)}'
for r in 1 2; do for th in 0 10; do
  YDBL_BNECK_TH=$th timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bth/bench_th${th}_r$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/bth/bench_th${th}_r$r.json
done; done
