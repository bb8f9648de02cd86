# Round 5: bench.py DBL-n bs32 with the class-split NMS (default) vs one workgroup per image (YDBL_NMS_GROUPS=0), alternating
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; set -o pipefail
for r in 1 2 3; do
  for v in groups single; do
    E=""; [ $v = single ] && E="YDBL_NMS_GROUPS=0"
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/nms_$v.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/nms_$v.json "$v r$r"
  done
done
