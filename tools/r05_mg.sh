#!/bin/bash
# conv1 XCD mask-group A/B at the large configs (tools/r05_mg.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=mvdet_amd/lib/exp/libmvbev_mg2.so,mvdet_amd/lib/exp/libmvbev_mg4.so,mvdet_amd/lib/exp/libmvbev_mg8.so
for c in 3 5; do
  timeout -k 10 400 python tools/kbench.py --config $c --only winoconv --libs $L --rounds 2 --reps 8 > gpurun_out/$1_cfg$c.jsonl 2> gpurun_out/$1_cfg$c.err || { tail -20 gpurun_out/$1_cfg$c.err; exit 1; }
  grep stage gpurun_out/$1_cfg$c.jsonl
done
