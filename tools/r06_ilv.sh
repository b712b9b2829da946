#!/bin/bash
# Round 6: interleaved MFMA order over the Cout blocks (MVBEV_WINO_ILV=1, bitwise the same sums) vs the default,
# (MVBEV_WINO_ILV was removed after this measurement: DESIGN.md §4)
# interleaved kbench at cfg2 / cfg3 (tools/r06_ilv.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in 2 3; do
  timeout -k 10 300 python -u tools/kbench.py --config $cfg --only winoconv,conv23w,winoconv43,conv2w43 --rounds 3 --reps 10 \
    --libs mvdet_amd/lib/exp/libmvbev_ilv.so >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
echo ilv-done
