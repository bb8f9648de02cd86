# One GPU iteration: the whole GPU suite, the default bench line (no CPU leg) and the in-graph bs16 layer profile.
# usage: bash scripts/gpu_iter.sh TAG [pytest -k expr]
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=${1:-it}; mkdir -p gpurun_out/$T
K=${2:+-k "$2"}
eval timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider $K \
  > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2>gpurun_out/$T/bench.err || exit 1
cut -c1-400 gpurun_out/$T/bench.json
timeout -k 10 200 python scripts/layer_profile.py --batch 16 > gpurun_out/$T/layers_bs16.txt 2>&1 || exit 1
head -16 gpurun_out/$T/layers_bs16.txt
