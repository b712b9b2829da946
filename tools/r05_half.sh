#!/bin/bash
# A/B of the two-workgroups-per-CU Winograd conv (tools/r05_half.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=mvdet_amd/lib/exp/libmvbev_half.so
MVBEV_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wino.py > gpurun_out/$1_pytest.txt 2>&1 || { tail -30 gpurun_out/$1_pytest.txt; exit 1; }
tail -1 gpurun_out/$1_pytest.txt
for c in 2 5; do
  timeout -k 10 300 python tools/kbench.py --config $c --only winoconv,conv23w --libs $L --rounds 3 --reps 10 > gpurun_out/$1_cfg$c.jsonl 2> gpurun_out/$1_cfg$c.err || { tail -20 gpurun_out/$1_cfg$c.err; exit 1; }
  grep stage gpurun_out/$1_cfg$c.jsonl
done
