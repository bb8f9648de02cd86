# HBM traffic counters for the bench workload (separate passes, --kernel-trace only; MI355X_MICROARCH.md
# rocprofv3 PMC section).  Usage on the GPU box: bash scripts/pmc.sh <tag>
cd ${GRAFT_REPO_ROOT:-.}; T=gpurun_out/${1:-pmc}; mkdir -p $T; export TMPDIR=/tmp
rocprofv3 -L > $T/counters_list.txt 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -f csv -d $T/$C -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $T/$C.log 2>&1 || { echo "pmc $C failed"; tail -20 $T/$C.log; exit 1; }
done
ls -R $T | head -30
