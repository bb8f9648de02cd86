cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03d; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "stem" > gpurun_out/r03d/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03d/pytest.log; [ $rc -eq 0 ] || exit $rc
for pc in 0 2 3 4 6 8; do YDBL_STEM2_PERSIST=$pc timeout -k 10 60 python scripts/stem2_bench.py 0 2>&1 | grep stem2 | sed "s/^/persist=$pc /"; done
YDBL_STEM2_TH=16 timeout -k 10 60 python scripts/stem2_bench.py 0 2>&1 | grep stem2 | sed "s/^/th16 persist=4 /"
YDBL_STEM2_TH=16 YDBL_STEM2_PERSIST=2 timeout -k 10 60 python scripts/stem2_bench.py 0 2>&1 | grep stem2 | sed "s/^/th16 persist=2 /"
YDBL_STEM2_TH=4 YDBL_STEM2_PERSIST=6 timeout -k 10 60 python scripts/stem2_bench.py 0 2>&1 | grep stem2 | sed "s/^/th4 persist=6 /"
