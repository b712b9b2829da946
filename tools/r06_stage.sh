#!/bin/bash
# Round 6: staging-box capacity of the NCHW fused warp (tools/r06_stage.sh TAG): kbench A/B of
# libmvbev variants built with -DMVBEV_WW_STAGE=640 / 1024 / 1536 against the default (384)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=mvdet_amd/lib/exp
for cfg in 2 5 3; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --only warpw0,warpw --rounds 3 --reps 20 \
    --libs $L/libmvbev_s640.so,$L/libmvbev_s1024.so,$L/libmvbev_s1536.so \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
cat gpurun_out/$1_kbench.jsonl
