#!/bin/bash
# 1-GPU gloo rehearsals of bench.py --gpus N (the multi-rank path, ranks sharing the box's GPU)
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/$1_gpus$n.json 2> gpurun_out/$1_gpus$n.err || exit $?
  tail -c 200 gpurun_out/$1_gpus$n.json
done
