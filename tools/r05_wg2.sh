#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad_wino.py > gpurun_out/$1_pytest_wino.txt 2>&1 || { tail -40 gpurun_out/$1_pytest_wino.txt; exit 1; }
tail -1 gpurun_out/$1_pytest_wino.txt
timeout -k 10 300 python tools/kbench.py --only wgrad2,wgrad2w --rounds 3 --reps 30 > gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
grep stage gpurun_out/$1_kbench.jsonl
bash tools/r05_train.sh $1
