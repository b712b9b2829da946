#!/bin/bash
# Round 6: counters of the NCHW fused warp at cfg3 (the north star's 480 x 1440 grid), where T's writes dominate
# (tools/r06_w3pmc.sh TAG)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for PMC in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc/$1_$i -o run -- \
    python3 tools/kbench.py --config 3 --only warpw --reps 2 > gpurun_out/pmc/$1_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc/$1_* > gpurun_out/pmc/$1_summary.txt && grep -A30 "warp_wino_kernel" gpurun_out/pmc/$1_summary.txt
