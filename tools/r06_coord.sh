#!/bin/bash
# Round 6: conv1's coord term as one VALU pass (ABI 12300) — parity (coord term, engine, one-call ABI, backward),
# then the training step (tools/r06_coord.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_bev_abi.py tests/test_gpu_backward.py tests/test_gpu_nonfinite.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -60 gpurun_out/$1_pytest.txt; exit 1; }
tail -3 gpurun_out/$1_pytest.txt
timeout -k 10 300 python -c "import json, bench; r = bench.run_train_step(2, 'bf16x3', 20, 5, False); print(json.dumps(r))" \
  > gpurun_out/$1_train.json 2> gpurun_out/$1_train.err || { tail -20 gpurun_out/$1_train.err; exit 1; }
