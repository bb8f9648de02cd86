# Same-box A/B of two whole trees (Python + library): abtmp/base (git archive of HEAD + its built library) vs the
# working tree; bench.py DBL-n bs32 default, three rounds alternating.  usage: bash scripts/gpu_tree_ab.sh TAG
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; set -o pipefail; T=$PWD/gpurun_out/$1; mkdir -p $T
for r in 1 2 3; do
  for v in base new; do
    D=$GRAFT_REPO_ROOT; [ $v = base ] && D=$GRAFT_REPO_ROOT/abtmp/base
    (cd $D && timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $T/bench_${v}_r$r.json 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $T/bench_${v}_r$r.json "bench $v r$r"
  done
done
