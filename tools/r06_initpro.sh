#!/bin/bash
# Round 6: the init term (conv1's coord term) folded into the row-Winograd convs' accumulators at their start
# instead of read in the epilogue — the whole GPU suite, then interleaved kbench against the previous build
# (mvdet_amd/lib/exp/libmvbev_base.so) at cfg2 / cfg3 / cfg5 (tools/r06_initpro.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
for cfg in 2 3 5; do
  timeout -k 10 300 python -u tools/kbench.py --config $cfg --only winoconv,winoconv43 --rounds 3 --reps 10 \
    --libs mvdet_amd/lib/exp/libmvbev_base.so >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
echo initpro-done
