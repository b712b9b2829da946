#!/bin/bash
# Round-5 GPU test session: the named GPU tests (default: the whole GPU suite) under their own time
# limits; output under gpurun_out/<tag>_pytest.txt.  Usage: tools/r05_tests.sh TAG [pytest args...]
mkdir -p gpurun_out
TAG=$1; shift
export TMPDIR=/tmp
ARGS=${@:-tests/}
timeout -k 10 1050 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu $ARGS > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.txt
exit $rc
