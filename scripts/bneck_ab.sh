cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/bn
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bottleneck" > gpurun_out/bn/t.log 2>&1; rc=$?; tail -3 gpurun_out/bn/t.log; [ $rc -eq 0 ] || exit $rc
for k in 0 1 2000; do echo "== th32 min $k"; YDBL_BNECK_TH32=$k timeout -k 10 120 python scripts/kbench.py "bneck c16@320" "bneck c32@160" 2>&1 | grep us/launch || exit 1; done
for k in 0 2000 1 0 2000 1; do YDBL_BNECK_TH32=$k timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bn/b$k.json 2>gpurun_out/bn/b$k.err || exit 1; echo "th32 min $k $(cut -c1-110 gpurun_out/bn/b$k.json | sed 's/.*"value"/value/')"; done
