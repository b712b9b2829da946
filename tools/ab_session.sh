#!/bin/bash
# A short GPU session: a subset of the GPU suite, then kbench stages (interleaved rounds).
# Usage: bash tools/ab_session.sh <tag> "<test files>" "<kbench stages>" [kbench extra args]
set -e
TAG=$1; TESTS=$2; STAGES=$3; shift 3
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS > gpurun_out/${TAG}_pytest.txt 2>&1
timeout -k 10 240 python tools/kbench.py --only $STAGES --rounds 3 --reps 30 "$@" > gpurun_out/${TAG}_kbench.jsonl
