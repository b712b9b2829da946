set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wino.py > gpurun_out/r04d_pytest.txt 2>&1
timeout -k 10 200 python tools/kbench.py --only warpw,warpwcl,warpupw --rounds 3 --reps 30 --libs mvdet_amd/lib/exp/libmvbev_pad4.so,mvdet_amd/lib/exp/libmvbev_pad8.so > gpurun_out/r04d_kbench.jsonl
