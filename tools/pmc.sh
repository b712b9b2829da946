#!/bin/bash
# Separate rocprofv3 --pmc passes over tools/kbench.py (one counter group per pass).
# Usage: bash tools/pmc.sh <tag> <stages> "<group1>" ["<group2>" ...]
# e.g.   bash tools/pmc.sh warp warp "TA_BUSY_avr TCP_TCC_READ_REQ_sum" "FETCH_SIZE"
set -o pipefail
TAG=$1; STAGES=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
i=0
for PMC in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $OUT/${TAG}_$i -o run -- \
    python3 tools/kbench.py --only $STAGES --reps 2 > $OUT/${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py $OUT/${TAG}_* > $OUT/${TAG}_summary.txt && cat $OUT/${TAG}_summary.txt
