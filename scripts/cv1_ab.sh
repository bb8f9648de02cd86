cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/cv1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dsc3k or dsconv or e2e_n640 or e2e_s640" > gpurun_out/cv1/t.log 2>&1; rc=$?; tail -3 gpurun_out/cv1/t.log; [ $rc -eq 0 ] || exit $rc
for k in 1 0 1 0 1 0; do if [ $k = 1 ]; then export YDBL_NO_CV1_FUSE=1; else unset YDBL_NO_CV1_FUSE; fi; timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/cv1/b$k.json 2>gpurun_out/cv1/b$k.err || exit 1; echo "nofuse=$k $(cut -c1-110 gpurun_out/cv1/b$k.json | sed 's/.*"value"/value/')"; done
unset YDBL_NO_CV1_FUSE
timeout -k 10 200 python scripts/layer_profile.py --batch 16 > gpurun_out/cv1/lp.txt 2>&1 || exit 1; head -2 gpurun_out/cv1/lp.txt; grep -E "Conv1x1x2|DSConv.k3s1" gpurun_out/cv1/lp.txt | head -8
for k in 1 0; do if [ $k = 1 ]; then export YDBL_NO_CV1_FUSE=1; else unset YDBL_NO_CV1_FUSE; fi; timeout -k 10 300 python bench.py --model s --batch 64 --no-cpu-baseline --no-roofline > gpurun_out/cv1/s$k.json 2>gpurun_out/cv1/s$k.err || exit 1; echo "s bs64 nofuse=$k $(cut -c1-110 gpurun_out/cv1/s$k.json | sed 's/.*"value"/value/')"; done
