cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03i; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "hypergraph or hyperace or c3ah" > gpurun_out/r03i/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03i/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03i/bench.log 2>&1; tail -1 gpurun_out/r03i/bench.log | cut -c1-200
timeout -k 10 150 python scripts/layer_profile.py --batch 16 > gpurun_out/r03i/layers_n16.txt 2>&1; grep -E "total|AdaHG" gpurun_out/r03i/layers_n16.txt
timeout -k 10 120 python scripts/kbench.py "hg " 2>&1 | grep us/launch
