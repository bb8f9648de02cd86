cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/halo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "halo or conv_dense or e2e_n640 or conv3x3" > gpurun_out/halo/t.log 2>&1; rc=$?; tail -3 gpurun_out/halo/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/kbench.py "conv 256->32" 2>&1 | grep us/launch
YDBL_HALO_TH=8 timeout -k 10 120 python scripts/kbench.py "conv 256->32" 2>&1 | grep us/launch
bash scripts/roofline_check.sh rfchk || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/halo/b$i.json 2>gpurun_out/halo/b$i.err || exit 1; cut -c1-120 gpurun_out/halo/b$i.json; done
