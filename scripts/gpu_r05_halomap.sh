# Round 5: halo-kernel staging lane maps (YDBL_HALO_MAP 0/1/2): parity of the halo conv tests under each map, kbench
# of the halo shapes (two rounds, alternating), and a TCP-access PMC pass per map.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05hm; mkdir -p $T
for m in 1 2; do
  YDBL_HALO_MAP=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "halo or fp8" > $T/pytest_map$m.log 2>&1 || { tail -20 $T/pytest_map$m.log; exit 1; }
  tail -1 $T/pytest_map$m.log
done
for r in 1 2; do for m in 0 1 2; do
  echo "== round $r map $m" >> $T/kbench.txt
  YDBL_HALO_MAP=$m timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" "k3s2@80 bs16" >> $T/kbench.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $T/kbench.txt
for m in 0 1 2; do
  YDBL_HALO_MAP=$m timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
    --kernel-trace -f csv -d $T/pm$m -o run -- python scripts/kbench.py "384->64 k3s1@40 bs16" --eager=20 > $T/pm$m.log 2>&1 || { echo "pmc $m failed"; tail -3 $T/pm$m.log; exit 1; }
done
python - $T <<'PY'
import csv, glob, sys, collections
for m in (0, 1, 2):
    agg = collections.defaultdict(list); dur = []
    for f in glob.glob(f"{sys.argv[1]}/pm{m}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "halo" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(f"{sys.argv[1]}/pm{m}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "halo" in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"map {m}: dur {sum(dur)/max(len(dur),1):.2f} us", {k: round(sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
timeout -k 10 900 python -u scripts/fp8_calibrate.py > $T/fp8_calibrate_task.txt 2>&1; rc=$?; tail -8 $T/fp8_calibrate_task.txt
cp tests/golden/fp8_calib_yolov13s_DBL_nc3.json $T/fp8_calib_task.json 2>/dev/null; exit $rc
