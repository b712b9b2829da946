#!/bin/bash
# Round 6: kernel traces of the training step with and without the SGD update, each in its own process
# (tools/r06_trainmode.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in no_update update no_update update; do
  timeout -k 10 200 python tools/train_mode.py $m 60 >> gpurun_out/$1_times.txt 2>> gpurun_out/$1.err || { tail -20 gpurun_out/$1.err; exit 1; }
done
cat gpurun_out/$1_times.txt
for m in no_update update; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof_$m -o run -- python tools/train_mode.py $m 60 \
    >> gpurun_out/$1.err 2>&1 || { tail -20 gpurun_out/$1.err; exit 1; }
done
find gpurun_out/$1_prof_* -name "*kernel_stats.csv" | sort
