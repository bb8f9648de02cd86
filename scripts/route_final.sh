cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 120 python scripts/kbench.py "conv 64->128 k1s1@80" "conv 128->64 k1s1@80" "conv 64->64 k3s2@80" "conv 64->128 k3s1@40" 2>&1 | grep us/launch || exit 1
for e in "X=1" "YDBL_IGEMM_R2=1 YDBL_HALO_N2=400" "X=1" "YDBL_IGEMM_R2=1 YDBL_HALO_N2=400"; do env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/route_b.json 2>/dev/null || exit 1; echo "$e $(cut -c1-110 gpurun_out/route_b.json | sed 's/.*"value"/value/')"; done
bash scripts/gpu_r03_final2.sh r03fin4
