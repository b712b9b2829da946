#!/bin/bash
# Round 6: the training warp adjoint (warp_adjoint_pix_kernel) — timing and separate PMC passes
# (tools/r06_adjpmc.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/kbench.py --config 2 --only adjpix,adjuppix --rounds 3 --reps 20 \
  > gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
cat gpurun_out/$1_kbench.jsonl
bash tools/pmc.sh $1 adjpix,adjuppix \
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
  "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
  "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR"
