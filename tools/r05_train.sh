#!/bin/bash
# backward suite + the bench's training-step lines (tools/r05_train.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_wgrad_wino.py > gpurun_out/$1_pytest_bwd.txt 2>&1 || { tail -40 gpurun_out/$1_pytest_bwd.txt; exit 1; }
tail -2 gpurun_out/$1_pytest_bwd.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --north-star-cfg 0 --roofline-cfg 0 --batch-cfg 0 --no-alt --no-probe > gpurun_out/$1_bench.json 2> gpurun_out/$1_bench.err || { tail -20 gpurun_out/$1_bench.err; exit 1; }
python - "$1" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}_bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"])
t = d.get("train_step", {})
print(json.dumps({k: t[k] for k in t if k in ("value", "ms_per_step", "stages_ms", "torch", "plus_a4")})[:1500])
PY
