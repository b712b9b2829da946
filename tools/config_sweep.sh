# Parity report (configs 1, 2, 4) and a short bench of configs 1, 3, 4, 5 on the GPU box;
# outputs under gpurun_out/sweep/.  Usage: bash tools/config_sweep.sh
set -o pipefail
mkdir -p gpurun_out/sweep
for c in 1 2 4; do
  timeout -k 10 200 python -u tools/parity_report.py --config $c --precision bf16x3 > gpurun_out/sweep/parity_$c.json 2>gpurun_out/sweep/parity_$c.err || exit 1
done
for c in 1 3 4 5; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-train --no-alt --steps 10 --warmup 3 > gpurun_out/sweep/bench_$c.json 2>gpurun_out/sweep/bench_$c.err || exit 1
done
echo sweep-done
