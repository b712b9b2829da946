#!/bin/bash
# Round-4 GPU session: the GPU suite, the bench, then A/B kernel timings (tools/kbench.py, separate
# processes per variant: the variant selections are read once per process).  Every GPU step has its
# own time limit.  Ordinary test failures (pytest rc 1) do not stop the session; a time limit, an
# abort or a crash does (nothing runs on the GPU after it), as does any failure of a later step.
mkdir -p gpurun_out
TAG=${1:-r04a}
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 420 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 120 python tools/kbench.py --only warpw,warpwcl --rounds 2 --reps 30 >> gpurun_out/${TAG}_kbench.jsonl
timeout -k 10 120 python tools/kbench.py --only warpupwn,warpupwt,warpupwcl,conv1,conv2 --rounds 2 --reps 30 >> gpurun_out/${TAG}_kbench.jsonl
timeout -k 10 120 python tools/kbench.py --only winoconv,conv23w --rounds 2 --reps 30 >> gpurun_out/${TAG}_kbench.jsonl
