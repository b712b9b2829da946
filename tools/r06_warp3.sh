#!/bin/bash
# Round 6: box tables of the channels-last warps — parity, then A/B timing (tools/r06_warp3.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_nonfinite.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -60 gpurun_out/$1_pytest.txt; exit 1; }
tail -3 gpurun_out/$1_pytest.txt
for cfg in 2 3; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --only warpupwcl0,warpupwcl,warpwcl0,warpwcl,warpw0,warpw --rounds 3 --reps 20 \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
cat gpurun_out/$1_kbench.jsonl
