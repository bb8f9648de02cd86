# Halo-kernel chunk prefetch depth (YDBL_HALO_PF): parity at 2 / 3, kbench conv cases, bench A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/hpf
for pf in 2 3; do
  YDBL_HALO_PF=$pf timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "conv3x3_halo or conv_fp8 or conv_dense" > gpurun_out/hpf/test_pf$pf.log 2>&1; rc=$?
  tail -1 gpurun_out/hpf/test_pf$pf.log; [ $rc -eq 0 ] || exit $rc
done
for pf in 1 2 3; do
  YDBL_HALO_PF=$pf timeout -k 10 300 python scripts/kbench.py "conv 384" "conv 256->" "conv 192" "conv 64->128 k3" "conv 128->128 k3" "conv 32->64 k3s1" "conv 64->64 k3s1" > gpurun_out/hpf/kb_pf$pf.txt 2>&1 || exit 1
done
paste gpurun_out/hpf/kb_pf1.txt gpurun_out/hpf/kb_pf2.txt gpurun_out/hpf/kb_pf3.txt | awk -F'\t' '{printf "%-44s %8s %8s %8s\n", substr($1,1,42), substr($1,42,9), substr($2,42,9), substr($3,42,9)}'
for r in 1 2; do for pf in 1 2; do
  YDBL_HALO_PF=$pf timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/hpf/bench_pf${pf}_r$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/hpf/bench_pf${pf}_r$r.json
done; done
