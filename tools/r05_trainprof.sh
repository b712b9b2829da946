#!/bin/bash
# kernel trace of the native training step (tools/r05_trainprof.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$1_trace -o run -- python3 $R/tools/train_bench.py --steps 12 --warmup 3 --no-torch > $R/gpurun_out/$1_trace.log 2>&1 || exit 1
tail -2 $R/gpurun_out/$1_trace.log
f=$(find $R/gpurun_out/$1_trace -name "*kernel_stats.csv" | head -1); head -40 $f | cut -c1-200
