#!/bin/bash
# Round 6: the F(4,3) conv's 8 x 64 tile mode (MVBEV_W43_TILES_8X64) — parity, then interleaved kbench of conv1 in
# (the wide-mode stages winoconv43w / conv2w43w and MVBEV_W43_TILES_8X64 were removed after this measurement: DESIGN.md §4)
# F(3,3), F(4,3) 16 x 32 and F(4,3) 8 x 64 at cfg1 / cfg2 (tools/r06_w43w.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wino43.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
for cfg in 2 1 4; do
  timeout -k 10 300 python -u tools/kbench.py --config $cfg --check43 \
    --only winoconv,winoconv43,winoconv43w,conv23w,conv23w43,conv2w43,conv2w43w --rounds 3 --reps 10 \
    >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
grep check43 gpurun_out/$1_kbench.jsonl
