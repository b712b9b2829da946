set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/train_trace -o run -- python3 tools/train_bench.py --config 2 --steps 10 --warmup 3 --no-torch > gpurun_out/prof/train_trace.log 2>&1 || exit $?
echo done
