#!/bin/bash
# verify the runtime mask group: full-size parity + conv1 timings at cfg2 / 4 / 5 (tools/r05_mgv.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_wino.py > gpurun_out/$1_pytest.txt 2>&1 || { tail -30 gpurun_out/$1_pytest.txt; exit 1; }
tail -1 gpurun_out/$1_pytest.txt
for c in 2 4 5; do
  timeout -k 10 300 python tools/kbench.py --config $c --only winoconv,conv23w --rounds 2 --reps 8 > gpurun_out/$1_cfg$c.jsonl 2> gpurun_out/$1_cfg$c.err || { tail -20 gpurun_out/$1_cfg$c.err; exit 1; }
  grep stage gpurun_out/$1_cfg$c.jsonl
done
