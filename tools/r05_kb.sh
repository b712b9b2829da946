#!/bin/bash
# kbench of the default library: tools/r05_kb.sh TAG STAGES [ROUNDS]
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py --only "$2" --rounds ${3:-3} --reps 30 > gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err
rc=$?
tail -c 300 gpurun_out/$1_kbench.err
exit $rc
