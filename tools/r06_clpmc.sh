#!/bin/bash
# Round 6: counters of the channels-last fused warps at cfg3 (tools/r06_clpmc.sh TAG)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for PMC in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc/$1_$i -o run -- \
    python3 tools/kbench.py --config 3 --only warpw,warpwcl,warpupwcl --reps 2 > gpurun_out/pmc/$1_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc/$1_* > gpurun_out/pmc/$1_summary.txt && grep -A22 "warp_wino_cl_kernel\|warp_up_wino_cl_kernel\|warp_wino_kernel<" gpurun_out/pmc/$1_summary.txt
