#!/bin/bash
# Round 6: the full default bench.py --gpus 8 flow (alternative modes, north-star cfg3, CPU baseline) as a
# 1-GPU gloo rehearsal (8 ranks sharing the box's GPU; tools/r06_rehearse8.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python bench.py --gpus 8 --steps 6 --warmup 2 > gpurun_out/$1_gpus8.json 2> gpurun_out/$1_gpus8.err || { tail -30 gpurun_out/$1_gpus8.err; exit 1; }
tail -c 400 gpurun_out/$1_gpus8.json
