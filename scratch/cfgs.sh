set -e
for c in 1 3 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-train --no-alt > gpurun_out/cfg$c.log 2>&1
done
MVBEV_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/mp2.log 2>&1
