# quick GPU pass: parity tests, per-launch profile, NMS micro-bench under rocprof (tag = $1)
cd $GRAFT_REPO_ROOT; T=gpurun_out/${1:-quick}; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $T/pytest_gpu.log 2>&1; rc=$?
tail -5 $T/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/layer_profile.py > $T/layers_n.txt 2>&1 && head -16 $T/layers_n.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $T/nmsprof -o nms -- python scripts/nms_bench.py > $T/nms.txt 2>&1; grep cands $T/nms.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $T/prof -o bench -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $T/bench.txt 2>&1; tail -1 $T/bench.txt
