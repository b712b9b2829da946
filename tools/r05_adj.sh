#!/bin/bash
# adjoint A/B + parity of the variant libs (tools/r05_adj.sh TAG LIBS)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py --only adj,adjup --libs "$2" --rounds 3 --reps 30 > gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
grep stage gpurun_out/$1_kbench.jsonl
for L in ${2//,/ }; do
  MVBEV_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_backward.py -k "adjoint or training_step" > gpurun_out/$1_pytest_$(basename $L .so).txt 2>&1 || { tail -30 gpurun_out/$1_pytest_$(basename $L .so).txt; exit 1; }
  tail -1 gpurun_out/$1_pytest_$(basename $L .so).txt
done
