#!/bin/bash
# Round 6: 2 channel groups per block at 7 waves with 32-bit staging offsets (in-tree build) — parity of the
# fused-warp suites, then kbench A/B against the previous build and the 64-bit-offset 2-group variant
# (tools/r06_groups2.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_nonfinite.py \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_bev_abi.py > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
L=mvdet_amd/lib/exp
for cfg in 3 2 5 4; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --only warpw --rounds 3 --reps 20 \
    --libs $L/libmvbev_base.so,$L/libmvbev_g2w7.so >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
