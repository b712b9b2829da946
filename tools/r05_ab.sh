#!/bin/bash
# A/B kernel timings (tools/kbench.py, interleaved rounds of the default library and the variants);
# usage: tools/r05_ab.sh TAG STAGES LIB[,LIB...]
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py --only "$2" --libs "$3" --rounds 3 --reps 30 > gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err
rc=$?
tail -c 400 gpurun_out/$1_kbench.err
exit $rc
