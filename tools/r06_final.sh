#!/bin/bash
# Round 6 (F(4,3) tree): the default bench line, then the rocprofv3 set — cfg2 kernel trace, PMC passes, traffic,
# cfg5 trace (tools/profile_gpu.sh), plus the cfg3 (north-star) kernel trace (tools/r06_final.sh TAG)
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/$1_bench.json 2> gpurun_out/$1_bench.err || { tail -30 gpurun_out/$1_bench.err; exit 1; }
tail -c 300 gpurun_out/$1_bench.json
bash tools/profile_gpu.sh $1 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$1_trace_cfg3 -o run -- \
  python3 bench.py --steps 5 --warmup 2 --config 3 --no-cpu-baseline --no-train --no-alt --no-probe --north-star-cfg 0 --batch-cfg 0 \
  --roofline-cfg 0 > gpurun_out/prof/$1_trace_cfg3_bench.log 2>&1 || exit 1
echo final-done
