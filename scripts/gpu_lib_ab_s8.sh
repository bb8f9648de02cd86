# Same-box A/B of the in-tree library vs abtmp/libydbl_base.so on the config-3 per-rank workload (DBL-s bs8)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
for r in 1 2; do
  for v in base new; do
    L=""; [ $v = base ] && L="YDBL_LIB=abtmp/libydbl_base.so"
    env $L timeout -k 10 200 python bench.py --model s --batch 8 --no-cpu-baseline --no-roofline > $T/s8_${v}_r$r.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $T/s8_${v}_r$r.json "DBL-s bs8 $v r$r"
  done
done
