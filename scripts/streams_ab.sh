cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for st in 1 2 3 4; do timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --streams $st 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams $st', d['value'], d['ms_per_step'])"; done
