#!/bin/bash
# Round 6: row-Winograd F(4,3), xi-major (ABI 12400) — parity vs float64 / F(3,3), full-size difference vs F(3,3),
# and interleaved kbench of the F(3,3) and F(4,3) conv1 / conv2 -> conv3 stages (tools/r06_w43.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wino43.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
for cfg in 2 3 5; do
  timeout -k 10 300 python -u tools/kbench.py --config $cfg --check43 \
    --only winoconv,winoconv43,conv23w,conv23w43,conv2w43,winorows2_43 --rounds 3 --reps 10 \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
grep check43 gpurun_out/$1_kbench.jsonl
