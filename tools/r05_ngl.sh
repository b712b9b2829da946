#!/bin/bash
# fused NCHW warp, several channel groups per block, at the large configs (tools/r05_ngl.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=mvdet_amd/lib/exp/libmvbev_ng1.so,mvdet_amd/lib/exp/libmvbev_ng2.so,mvdet_amd/lib/exp/libmvbev_ng4.so
for c in 3 5 2; do
  timeout -k 10 300 python tools/kbench.py --config $c --only warpw --libs $L --rounds 2 --reps 10 > gpurun_out/$1_cfg$c.jsonl 2> gpurun_out/$1_cfg$c.err || { tail -20 gpurun_out/$1_cfg$c.err; exit 1; }
  grep stage gpurun_out/$1_cfg$c.jsonl
done
