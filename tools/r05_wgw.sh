#!/bin/bash
# Winograd conv1 wgrad: parity tests, backward suite, kernel timing (tools/r05_wgw.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad_wino.py > gpurun_out/$1_pytest_wino.txt 2>&1 || { tail -40 gpurun_out/$1_pytest_wino.txt; exit 1; }
tail -3 gpurun_out/$1_pytest_wino.txt
timeout -k 10 300 python tools/kbench.py --only wgrad1,wgrad1w --rounds 3 --reps 30 > gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
cat gpurun_out/$1_kbench.jsonl | tail -6
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_backward.py > gpurun_out/$1_pytest_bwd.txt 2>&1 || { tail -40 gpurun_out/$1_pytest_bwd.txt; exit 1; }
tail -3 gpurun_out/$1_pytest_bwd.txt
