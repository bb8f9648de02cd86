# Round 5: memory-path probe of the deep-K halo 3x3 convs.  (1) scripts/bin/l2_probe: per-CU read bandwidth from
# L2 / MALL / HBM at the halo kernel's occupancy and loads in flight; (2) kbench in-graph times of the halo shapes;
# (3) per-kernel PMC passes (TCP/TCC/TA/TD/SQ) over those shapes (kernel-trace only, one group per pass).
# usage: bash scripts/gpu_r05_memprobe.sh TAG
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 120 scripts/bin/l2_probe > $T/l2_probe.txt 2>&1 || exit 1
cat $T/l2_probe.txt
timeout -k 10 200 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" "k3s1@20 bs16" > $T/kbench_halo.txt 2>&1 || exit 1
cat $T/kbench_halo.txt
i=0
for C in "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
         "TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -f csv -d $T/p$i -o run -- python scripts/kbench.py "k3s1@40 bs16" "256->32 k3s1@80 bs16" --eager=20 \
    > $T/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $T/p$i.log; exit 1; }
done
python - $T <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ydbl" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:36s} {sum(v) / len(v):16.0f}  (n={len(v)})")
PY
# halo tile-height / channel-slice A/B on the deep-K head 3x3 shapes (bs16 sub-batch graphs), two rounds
for r in 1 2; do
  for e in "-" "YDBL_HALO_TH=16" "YDBL_HALO_TH=20" "YDBL_HALO_TH=8 YDBL_HALO_NTN=4" "YDBL_HALO_TH=16 YDBL_HALO_NTN=4"; do
    echo "== round $r env $e" >> $T/halo_ab.txt
    if [ "$e" = "-" ]; then timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/halo_ab.txt 2>&1 || exit 1
    else env $e timeout -k 10 120 python scripts/kbench.py "k3s1@40 bs16" "k3s1@80 bs16" >> $T/halo_ab.txt 2>&1 || exit 1; fi
  done
done
cat $T/halo_ab.txt
