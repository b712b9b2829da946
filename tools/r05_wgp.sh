#!/bin/bash
# Winograd wgrad partition sweep + kernel trace (tools/r05_wgp.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 1 2 4 8; do
  MVBEV_WGRAD_WINO_P=$P timeout -k 10 200 python tools/kbench.py --only wgrad1w --rounds 2 --reps 30 > gpurun_out/$1_P$P.jsonl 2> gpurun_out/$1_P$P.err || exit 1
  echo P=$P; grep '"stage"' gpurun_out/$1_P$P.jsonl
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$1_prof -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --only wgrad1w --rounds 1 --reps 20 > $GRAFT_REPO_ROOT/gpurun_out/$1_prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/$1_prof -name "*kernel_stats.csv" | head -1 | xargs head -12
