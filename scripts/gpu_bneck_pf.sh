# Persistent Bottleneck walk: parity, phase stamps, kbench, layer profile, bench.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/bpf
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "bottleneck or detect_box" > gpurun_out/bpf/test.log 2>&1; rc=$?; tail -1 gpurun_out/bpf/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py bneck box3 > gpurun_out/bpf/kb.txt 2>&1 || exit 1
cat gpurun_out/bpf/kb.txt | grep -v amdgpu.ids
bash scripts/build_stamps.sh bneck > /dev/null 2>&1 && timeout -k 10 200 python scripts/bneck_stamps.py > gpurun_out/bpf/stamps.txt 2>&1; cat gpurun_out/bpf/stamps.txt | grep -v amdgpu.ids
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bpf/bench_r$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/bpf/bench_r$r.json
done
