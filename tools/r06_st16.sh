#!/bin/bash
# Round 6: the NCHW fused warps' phase 2 with one 16-B T store per lane and row (lane pairs; MVBEV_WW_STORE16) —
# parity of the warp / nonfinite / fullsize suites, then interleaved kbench against the 4-B-store build
# (mvdet_amd/lib/exp/libmvbev_base.so) at cfg2 / cfg3 / cfg5 (tools/r06_st16.sh TAG)
# (MVBEV_WW_STORE16 was removed after this measurement: 16-B stores ran 1-3.5 % slower)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_wino43.py \
  tests/test_gpu_nonfinite.py tests/test_gpu_fullsize.py > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
for cfg in 2 3 5; do
  timeout -k 10 300 python -u tools/kbench.py --config $cfg --only warpw,warpw43 --rounds 3 --reps 10 \
    --libs mvdet_amd/lib/exp/libmvbev_base.so >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
echo st16-done
