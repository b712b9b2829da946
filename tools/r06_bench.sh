#!/bin/bash
# Round 6: the default bench line (tools/r06_bench.sh TAG [extra bench args])
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 1100 python bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
tail -c 300 gpurun_out/${tag}_bench.json
