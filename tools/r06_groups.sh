#!/bin/bash
# Round 6: several 8-channel groups per block of the NCHW fused warp (cfg3: ~480 instructions per wave of block
# setup around 8 channels' work) — parity of the in-tree build (4 groups), then kbench A/B of group / occupancy
# variants (tools/r06_groups.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_nonfinite.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
L=mvdet_amd/lib/exp
for cfg in 3 2 5; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --only warpw --rounds 3 --reps 20 \
    --libs $L/libmvbev_base.so,$L/libmvbev_g1w8.so,$L/libmvbev_g2w7.so,$L/libmvbev_g2w8.so,$L/libmvbev_g4w6.so \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
