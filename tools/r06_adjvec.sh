#!/bin/bash
# Round 6: 16-B stores in the warp adjoint (warp_adjoint_pix_kernel; TD 91 % busy with 7.3 M dword store
# instructions per launch): backward parity, kbench A/B against mvdet_amd/lib/exp/libmvbev_base.so, training step
# (tools/r06_adjvec.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_backward.py \
  > gpurun_out/$1_pytest.txt 2>&1 || { tail -60 gpurun_out/$1_pytest.txt; exit 1; }
tail -3 gpurun_out/$1_pytest.txt
timeout -k 10 200 python tools/kbench.py --config 2 --only adjpix,adjuppix --rounds 3 --reps 20 \
  --libs mvdet_amd/lib/exp/libmvbev_base.so > gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
cat gpurun_out/$1_kbench.jsonl
bash tools/pmc.sh $1 adjpix,adjuppix "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" > /dev/null
cat gpurun_out/pmc/$1_summary.txt
timeout -k 10 300 python -c "import json, bench; r = bench.run_train_step(2, 'bf16x3', 20, 5, False); print(json.dumps(r))" \
  > gpurun_out/$1_train.json 2> gpurun_out/$1_train.err || { tail -20 gpurun_out/$1_train.err; exit 1; }
