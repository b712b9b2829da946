#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
L=mvdet_amd/lib/exp/libmvbev_s4.so
for c in 2 5 3 4; do
  timeout -k 10 300 python tools/kbench.py --config $c --only winoconv --libs $L --rounds 3 --reps 8 > gpurun_out/$1_cfg$c.jsonl 2> gpurun_out/$1_cfg$c.err || { tail -20 gpurun_out/$1_cfg$c.err; exit 1; }
  grep stage gpurun_out/$1_cfg$c.jsonl
done
