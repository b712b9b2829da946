#!/bin/bash
# Round 6 (F(4,3) tree): 1-GPU rehearsals of bench.py --gpus 2 and --gpus 8 (ranks sharing the box's GPU)
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 8; do
  timeout -k 10 500 python bench.py --gpus $n --steps 6 --warmup 2 > gpurun_out/$1_gpus$n.json 2> gpurun_out/$1_gpus$n.err \
    || { tail -30 gpurun_out/$1_gpus$n.err; exit 1; }
  tail -c 400 gpurun_out/$1_gpus$n.json; echo
done
