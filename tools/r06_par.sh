#!/bin/bash
# Round 6: the multi-rank path with the channel-slice exchange (tools/r06_par.sh TAG):
# the multi-GPU GPU tests (gloo ranks sharing the box's GPU; one-rank RCCL pipelines), then
# 1-GPU gloo rehearsals of bench.py --gpus 2 / 8 at cfg2 (8 ranks: the channel parts + fetch of the node)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parallel.py ${PYK:+-k "$PYK"} \
  > gpurun_out/$1_pytest_parallel.txt 2>&1 || { tail -60 gpurun_out/$1_pytest_parallel.txt; exit 1; }
tail -3 gpurun_out/$1_pytest_parallel.txt
for n in 2 8; do
  timeout -k 10 500 python bench.py --gpus $n --steps 6 --warmup 2 --no-cpu-baseline --no-alt \
    > gpurun_out/$1_gpus$n.json 2> gpurun_out/$1_gpus$n.err || { tail -30 gpurun_out/$1_gpus$n.err; exit 1; }
  tail -c 600 gpurun_out/$1_gpus$n.json
done
