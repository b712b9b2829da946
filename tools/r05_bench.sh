#!/bin/bash
# the default bench line, timed (tools/r05_bench.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/$1_bench.json 2> gpurun_out/$1_bench.err
rc=$?
echo "bench rc=$rc wall=$(( $(date +%s) - t0 ))s"
tail -c 400 gpurun_out/$1_bench.err
exit $rc
