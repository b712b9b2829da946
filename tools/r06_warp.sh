#!/bin/bash
# Round 6: the fused warp's per-geometry box table — parity tests, then interleaved timing (tools/r06_warp.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_rows.py \
  > gpurun_out/$1_pytest_wino.txt 2>&1 || { tail -60 gpurun_out/$1_pytest_wino.txt; exit 1; }
tail -3 gpurun_out/$1_pytest_wino.txt
for cfg in 2 3 5; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --only warpw0,warpw --rounds 3 --reps 20 \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
cat gpurun_out/$1_kbench.jsonl
