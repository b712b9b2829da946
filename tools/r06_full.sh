#!/bin/bash
# Round 6: the default N=1 bench line, then a full-default 1-GPU gloo rehearsal of bench.py --gpus 4 (tools/r06_full.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python bench.py > gpurun_out/$1_bench.json 2> gpurun_out/$1_bench.err || { tail -30 gpurun_out/$1_bench.err; exit 1; }
tail -c 200 gpurun_out/$1_bench.json
timeout -k 10 900 python bench.py --gpus 4 --steps 8 --warmup 2 > gpurun_out/$1_gpus4.json 2> gpurun_out/$1_gpus4.err || { tail -30 gpurun_out/$1_gpus4.err; exit 1; }
tail -c 300 gpurun_out/$1_gpus4.json
