#!/bin/bash
# Round 6: training-path GPU tests (non-finite guard, backward suite), then the default bench (tools/r06_train.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nonfinite.py \
  > gpurun_out/$1_pytest_nonfinite.txt 2>&1 || { tail -60 gpurun_out/$1_pytest_nonfinite.txt; exit 1; }
tail -3 gpurun_out/$1_pytest_nonfinite.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_backward.py \
  > gpurun_out/$1_pytest_bwd.txt 2>&1 || { tail -60 gpurun_out/$1_pytest_bwd.txt; exit 1; }
tail -3 gpurun_out/$1_pytest_bwd.txt
if [ -z "$NOBENCH" ]; then
  timeout -k 10 1100 python bench.py > gpurun_out/$1_bench.json 2> gpurun_out/$1_bench.err || { tail -30 gpurun_out/$1_bench.err; exit 1; }
  tail -c 300 gpurun_out/$1_bench.json
fi
