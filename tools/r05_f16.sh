#!/bin/bash
# fp16 fused-warp checks + the cfg4 line (tools/r05_f16.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows.py "tests/test_gpu_fullsize.py::test_config4_fp16_batch8_vs_oracle_bands" > gpurun_out/$1_pytest.txt 2>&1 || { tail -30 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
timeout -k 10 400 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --north-star-cfg 0 --roofline-cfg 0 --batch-cfg 0 --no-train --no-alt --no-probe > gpurun_out/$1_bench4.json 2> gpurun_out/$1_bench4.err || { tail -20 gpurun_out/$1_bench4.err; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/$1_bench4.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stages_ms'])"
