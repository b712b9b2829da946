#!/bin/bash
# Round-5 GPU session: selected GPU tests, then the default bench line (each step under its own limit;
# nothing runs on the GPU after a step that timed out, aborted or crashed).
mkdir -p gpurun_out
TAG=$1; shift
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu "$@" > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 540 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc2=$?
tail -c 600 gpurun_out/${TAG}_bench.err
exit $(( rc > rc2 ? rc : rc2 ))
