#!/bin/bash
# Round 6: the whole GPU suite, smoke(), then a kernel trace of the training step (tools/r06_suite.sh TAG)
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -m gpu -v --timeout 400 --timeout-method thread tests > gpurun_out/$1_pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/$1_pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$1_smoke.txt 2>&1 || { cat gpurun_out/$1_smoke.txt; exit 1; }
cat gpurun_out/$1_smoke.txt
if [ -n "$TRACE" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$1_train -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-probe --north-star-cfg 0 --roofline-cfg 0 --batch-cfg 0 --train-torch 0 \
  > gpurun_out/$1_train_trace.log 2>&1 || { tail -20 gpurun_out/$1_train_trace.log; exit 1; }
fi
exit $rc
