# Round 5: XCD-aware tile order for every grid size (common.hpp xcd_remap / xcd_tile2): parity of the conv-family
# ops, same-box A/B against the previous library (abtmp/libydbl_base.so), then the per-launch conv fetch table.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r05xcd; mkdir -p $T
PARITY="conv or dsc or dysample or stem or lsk or bneck or halo or box3" bash scripts/gpu_lib_ab.sh r05xcd "conv" "dysample" "stem2" "bneck" > $T/ab.txt 2>&1 || { tail -30 $T/ab.txt; exit 1; }
cat $T/ab.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $T/fetch -o run -- python scripts/pmc_conv_fetch.py run $T/conv_steps.json > $T/fetch.log 2>&1 || { tail -5 $T/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $T/write -o run -- python scripts/pmc_conv_fetch.py run $T/conv_steps.json > $T/write.log 2>&1 || { tail -5 $T/write.log; exit 1; }
python scripts/pmc_conv_fetch.py report $T/conv_steps.json $T/fetch $T/write > $T/conv_fetch_table.txt 2>&1; tail -40 $T/conv_fetch_table.txt
