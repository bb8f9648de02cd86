# Bench A/B over environment settings: bash scripts/gpu_ab_env.sh TAG "ENV1" "ENV2" ... (each "K=V K2=V2" or "-")
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=$1; shift; mkdir -p gpurun_out/$T
for r in 1 2; do i=0; for e in "$@"; do i=$((i+1))
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/$T/bench_${i}_r$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/$T/bench_${i}_r$r.json "[$e]"
done; done
