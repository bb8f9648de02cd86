cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
C='conv 64->128 k3s1@40 bs16|conv 192->64 k3s1@40|conv 32->64 k3s1@80|conv 128->128 k3s2@40|conv 384->64 k3s1@40|conv 64->64 k3s2@80|conv 16->32 k3s2@320'
for e in "X=1" "YDBL_IGEMM_R2=1 YDBL_HALO_N2=400"; do
  echo "== $e"; env $e timeout -k 10 120 python scripts/kbench.py "conv 64->128 k3s1@40" "conv 192->64 k3s1@40" "conv 32->64 k3s1@80" "conv 128->128 k3s2@40" "conv 384->64 k3s1@40" "conv 64->64 k3s2@80" "conv 16->32 k3s2@320" "conv 128->64 k1s1@80" "conv 64->128 k1s1@80" "conv 64->128 k1s1@40" "conv 512->128 k1s1@40" "conv 256->64 k3s1@20" 2>&1 | grep us/launch || exit 1
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv or e2e_n640" > gpurun_out/route_t.log 2>&1; rc=$?; tail -1 gpurun_out/route_t.log; [ $rc -eq 0 ] || exit $rc
for e in "X=1" "YDBL_IGEMM_R2=1 YDBL_HALO_N2=400" "X=1" "YDBL_IGEMM_R2=1 YDBL_HALO_N2=400" "X=1" "YDBL_IGEMM_R2=1 YDBL_HALO_N2=400"; do env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/route_b.json 2>/dev/null || exit 1; echo "$e $(cut -c1-110 gpurun_out/route_b.json | sed 's/.*"value"/value/')"; done
for e in "X=1" "YDBL_IGEMM_R2=1 YDBL_HALO_N2=400"; do env $e timeout -k 10 300 python bench.py --model s --batch 64 --no-cpu-baseline --no-roofline > gpurun_out/route_s.json 2>/dev/null || exit 1; echo "s64 $e $(cut -c1-110 gpurun_out/route_s.json | sed 's/.*"value"/value/')"; done
