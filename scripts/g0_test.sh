cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "g0 or dsc3k" 2>&1 | tail -3
