#!/bin/bash
# Round 6: the split-output store's half-wave exchange as v_permlane32_swap instead of two ds_bpermute shuffles —
# the Winograd / BEV / parity suites, then interleaved kbench against HEAD's build
# (mvdet_amd/lib/exp/libmvbev_base.so) at cfg2 / cfg3 (tools/r06_perm.sh TAG)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_wino.py tests/test_gpu_wino43.py tests/test_gpu_bev_abi.py tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py > gpurun_out/$1_pytest.txt 2>&1 || { tail -40 gpurun_out/$1_pytest.txt; exit 1; }
tail -2 gpurun_out/$1_pytest.txt
for cfg in 2 3; do
  timeout -k 10 300 python -u tools/kbench.py --config $cfg --only winoconv,winoconv43,conv23w,conv23w43 --rounds 3 --reps 10 \
    --libs mvdet_amd/lib/exp/libmvbev_base.so >> gpurun_out/$1_kbench.jsonl 2> gpurun_out/$1_kbench.err || { tail -20 gpurun_out/$1_kbench.err; exit 1; }
done
echo perm-done
