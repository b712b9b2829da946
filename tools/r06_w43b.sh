#!/bin/bash
# Round 6: F(4,3) in the engine (fused warps writing T43, conv1 / conv2 -> conv3 F(4,3) where wino43_pays) — the
# wino / fullsize / nonfinite / parity suites, then a bench run without the CPU baseline (tools/r06_w43b.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wino43.py \
  tests/test_gpu_wino.py tests/test_gpu_fullsize.py tests/test_gpu_nonfinite.py tests/test_gpu_parity.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -60 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
timeout -k 10 600 python bench.py --no-cpu-baseline --no-alt --no-train > gpurun_out/$1_bench.json 2> gpurun_out/$1_bench.err \
  || { tail -30 gpurun_out/$1_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/$1_bench.json'))
print('cfg2', d['value'], d['stages_ms'])
for c in ('cfg3','cfg5','cfg4'):
    s=d.get(c) or {}; print(c, s.get('value'), s.get('stages_ms'))
"
