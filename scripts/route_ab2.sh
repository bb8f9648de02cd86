cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for e in "X=1" "YDBL_IGEMM_WANT=256" "YDBL_IGEMM_WANT=1024" "YDBL_IGEMM_BN64=0"; do
  echo "== $e"; env $e timeout -k 10 120 python scripts/kbench.py "conv 512->128 k1s1@40" "conv 384->128 k1s1@40" "conv 320->128 k1s1@40" "conv 128->192 k1s1@40" "conv 128->128 k1s1@40" "conv 384->256 k1s1@20" "conv 128->256 k1s1@20" "conv 256->128 k1s1@20" "conv 64->64 k3s1@20" "conv 16->32 k3s2@320" "conv 32->64 k3s2@160" "conv 128->128 k3s2@40" 2>&1 | grep us/launch || exit 1
done
