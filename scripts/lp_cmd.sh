cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/lp
timeout -k 10 200 python scripts/layer_profile.py --batch 16 > gpurun_out/lp/n16.txt 2>&1 || { tail gpurun_out/lp/n16.txt; exit 1; }
head -30 gpurun_out/lp/n16.txt
