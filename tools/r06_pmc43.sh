#!/bin/bash
# Round 6: PMC passes over the F(4,3) kernels at cfg5 (the BASELINE rocprof roofline config) -> their per-launch
# HBM traffic (traffic_cfg5_bf16x3_wino.json, read by bench.py's cfg5 sub-object), and an interleaved kbench of
# the F(3,3) / F(4,3) fused warps at cfg3 / cfg5 (tools/r06_pmc43.sh TAG)
OUT=gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for PMC in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
           "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $PMC --output-format csv -d $OUT/$1_pmc$i -o run -- \
    python3 tools/kbench.py --config 5 --reps 2 --only warpw43,winoconv43,conv2w43,winorows2_43 > $OUT/$1_pmc$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT/$1_pmc* > $OUT/$1_pmc_summary.txt
python3 tools/traffic.py $OUT $1 5 bf16x3 wino43 > $OUT/$1_traffic.json
for cfg in 3 5; do
  timeout -k 10 300 python -u tools/kbench.py --config $cfg --only warpw,warpw43 --rounds 3 --reps 10 \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
echo pmc43-done
