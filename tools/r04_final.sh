#!/bin/bash
# End-of-round GPU session: the GPU suite, smoke, the bench, a kernel trace of the training step.
set -e
mkdir -p gpurun_out
TAG=${1:-r04f}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
timeout -k 10 420 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trprof -o tr -- python -c "import bench; print(bench.run_train_step(2, 'bf16x3', 10, 2, with_torch=False))" > gpurun_out/${TAG}_trprof.log 2>&1
