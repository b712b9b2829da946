#!/bin/bash
# Round 6: the one-call path with F(4,3) (bev ABI tests, wino43 tests), then the MVBEV_WINO_ILV A/B (tools/r06_bev43.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bev_abi.py tests/test_gpu_wino43.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
bash tools/r06_ilv.sh $1
