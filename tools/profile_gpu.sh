#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root):
#   1. kernel trace + stats of bench.py (per-kernel durations)      -> gpurun_out/prof/<tag>_trace
#   2. separate --pmc passes on tools/kbench.py over the measured path's kernels (clock, MFMA
#      busy, HBM-side bytes, L2 hits, TA/TD load-path busy, stalls)
# Usage: bash tools/profile_gpu.sh <tag> [config]
set -o pipefail
TAG=${1:-r03}
CFG=${2:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_trace -o run -- \
  python3 bench.py --steps 10 --warmup 3 --config $CFG --no-cpu-baseline --no-train --no-alt --no-probe --north-star-cfg 0 --roofline-cfg 0 --batch-cfg 0 \
  > $OUT/${TAG}_trace_bench.log 2>&1 || exit $?
i=0
for PMC in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
           "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $OUT/${TAG}_pmc$i -o run -- \
    python3 tools/kbench.py --config $CFG --reps 3 --only warpw,warpwcl,warpupw,winoconv,conv23w > $OUT/${TAG}_pmc$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT/${TAG}_pmc* > $OUT/${TAG}_pmc_summary.txt
python3 tools/traffic.py $OUT $TAG $CFG bf16x3 wino > $OUT/${TAG}_traffic.json
# the kernel trace of the BASELINE "rocprof roofline run" config (cfg5: 8 views at 4K -> 1000 x 1000)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_trace_cfg5 -o run -- \
  python3 bench.py --steps 5 --warmup 2 --config 5 --no-cpu-baseline --no-train --no-alt --no-probe --north-star-cfg 0 --batch-cfg 0 \
  --roofline-cfg 0 > $OUT/${TAG}_trace_cfg5_bench.log 2>&1 || exit $?
echo profile-done
