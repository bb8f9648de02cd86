cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
echo "== default"; timeout -k 10 120 python scripts/kbench.py "conv 256->32" "conv 384" "conv 192" "conv 64->128 k3" "conv 32->64 k3s1" 2>&1 | grep us/launch
for th in 16 4; do echo "== th $th"; YDBL_HALO_TH=$th timeout -k 10 120 python scripts/kbench.py "conv 256->32" "conv 384" "conv 192" 2>&1 | grep us/launch; done
echo "== n2 off"; YDBL_HALO_N2=0 timeout -k 10 120 python scripts/kbench.py "conv 256->32" "conv 384" "conv 192" 2>&1 | grep us/launch
