#!/bin/bash
# Round 6: instruction mix of the Winograd convs at cfg2 (tools/r06_convpmc.sh TAG)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for PMC in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc/$1_$i -o run -- \
    python3 tools/kbench.py --config 2 --only winoconv,conv23w --reps 2 > gpurun_out/pmc/$1_$i.log 2>&1 || { echo "pass $i failed"; cat gpurun_out/pmc/$1_$i.log | tail -5; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc/$1_* > gpurun_out/pmc/$1_summary.txt && grep -A18 "conv_wino_kernel" gpurun_out/pmc/$1_summary.txt
