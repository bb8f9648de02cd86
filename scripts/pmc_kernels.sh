#!/bin/bash
# PMC counters per kernel for the kbench cases (one counter group per rocprofv3 pass, --kernel-trace only, each
# pass under its own hard timeout).  Usage on the GPU box: bash scripts/pmc_kernels.sh TAG [kbench case filters...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
T=gpurun_out/$TAG; mkdir -p $T; export TMPDIR=/tmp
CMD="python scripts/kbench.py --eager=3 $*"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -f csv -d $T/p$i -o run -- $CMD > $T/p$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -5 $T/p$i.log; exit 1; }
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -f csv -d $T/kt -o run -- $CMD > $T/kt.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
