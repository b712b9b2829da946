#!/bin/bash
# Round 6: the fused warps' scalar-instruction diet (fast block-index division, channel planes stepped instead of
# multiplied; cfg3 PMC: 1.9 G SALU vs 1.8 G VALU per launch) — parity, kbench A/B against libmvbev_base, SALU
# counters at cfg3 (tools/r06_salu.sh TAG)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_nonfinite.py \
  tests/test_gpu_fullsize.py > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
for cfg in 3 2 5; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --only warpw,warpwcl,warpupwcl --rounds 3 --reps 20 \
    --libs mvdet_amd/lib/exp/libmvbev_base.so >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv \
  -d gpurun_out/pmc/$1_1 -o run -- python3 tools/kbench.py --config 3 --only warpw --reps 2 > gpurun_out/pmc/$1_1.log 2>&1 || { echo "pmc failed"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc/$1_1 > gpurun_out/pmc/$1_summary.txt && grep -A7 "warp_wino_kernel" gpurun_out/pmc/$1_summary.txt
