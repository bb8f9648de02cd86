# Block-GEMM prefetch ring (YDBL_IGEMM_PF) + DSC3k chain: parity at PF 1 / 3, kbench conv cases at PF 1-4,
# in-graph layer profiles and bench A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pf
for pf in 1 3; do
  YDBL_IGEMM_PF=$pf timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "conv_dense or conv1x1 or conv3x3_halo or conv_fp8 or fullpad_fused_into_conv or blocks or chain" \
    > gpurun_out/pf/test_pf$pf.log 2>&1; rc=$?; tail -2 gpurun_out/pf/test_pf$pf.log; [ $rc -eq 0 ] || exit $rc
done
for pf in 1 2 3 4; do
  YDBL_IGEMM_PF=$pf timeout -k 10 300 python scripts/kbench.py conv > gpurun_out/pf/kb_pf$pf.txt 2>&1 || exit 1
done
paste gpurun_out/pf/kb_pf1.txt gpurun_out/pf/kb_pf3.txt | awk -F'\t' '{print substr($1,1,52), substr($2,42,9)}'
for cfg in "1 1" "3 1" "3 0"; do set -- $cfg
  YDBL_IGEMM_PF=$1 YDBL_DSC3K_CHAIN=$2 timeout -k 10 200 python scripts/layer_profile.py --batch 16 > gpurun_out/pf/layers_pf$1_chain$2.txt 2>&1 || exit 1
  head -2 gpurun_out/pf/layers_pf$1_chain$2.txt | tail -1
done
for r in 1 2; do for cfg in "1 1" "3 1" "3 0" "2 1"; do set -- $cfg
  YDBL_IGEMM_PF=$1 YDBL_DSC3K_CHAIN=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/pf/bench_pf$1_c$2_r$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/pf/bench_pf$1_c$2_r$r.json
done; done
