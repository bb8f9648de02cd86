# Per-kernel PMC probe of kbench shapes (one counter group per rocprofv3 --kernel-trace run, each under its own
# timeout), to see what bounds them: LDS vs VALU vs MFMA issue.  usage: bash scripts/gpu_pmc_probe.sh TAG "kbench filter"
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -s KILL 60 rocprofv3 -L > $T/avail.txt 2>&1 || true
i=0
for C in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
         "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -f csv -d $T/p$i -o run -- python scripts/kbench.py "$2" --eager=20 \
    > $T/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $T/p$i.log; }
done
ls -R $T | head -30
