# Round 5: the default bench line and the predict() line, three alternating runs each on one box (spread of the
# final numbers within a box; bench.py DBL-n bs32 fp16, no CPU leg / roofline).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; set -o pipefail; T=gpurun_out/r05rep; mkdir -p $T
for r in 1 2 3; do
  for m in session predict; do
    A=""; [ $m = predict ] && A="--via-predict"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $A > $T/${m}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $T/${m}_$r.json "$m r$r"
  done
done
