#!/bin/bash
# Round 6: pair-pass staging of the NCHW fused warp's large boxes (tools/r06_passes.sh TAG): the fused-warp
# parity tests, then kbench A/B against the previous build (mvdet_amd/lib/exp/libmvbev_base.so)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wino.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -60 gpurun_out/$1_pytest.txt; exit 1; }
tail -3 gpurun_out/$1_pytest.txt
for cfg in 2 5 3; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --only warpw --rounds 3 --reps 20 \
    --libs mvdet_amd/lib/exp/libmvbev_base.so \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
cat gpurun_out/$1_kbench.jsonl
