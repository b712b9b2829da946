#!/bin/bash
# One PMC pass (L2 -> fabric read requests, L2 hits/misses) of tools/kbench.py's stage $2 for each
# library variant given after it, each in its own rocprofv3 run (MVBEV_LIB selects the library).
# Usage: bash tools/pmc_ab.sh <tag> <stage> <lib> [<lib> ...]   (on the GPU box, from the repo root)
# PMC="<counters>" replaces the default counter set (one pass: mind the per-block slot limits).
set -o pipefail
TAG=$1; STAGE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for LIB in "$@"; do
  N=$(basename $LIB .so)
  MVBEV_LIB=$R/$LIB timeout -k 10 120 rocprofv3 --pmc ${PMC:-TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_HIT_sum TCC_MISS_sum} \
    --output-format csv -d $OUT/${TAG}_$N -o run -- python3 tools/kbench.py --config 2 --reps 3 --only $STAGE \
    > $OUT/${TAG}_$N.log 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT/${TAG}_$N > $OUT/${TAG}_${N}_summary.txt || exit $?
done
echo pmc-ab-done
