#!/bin/bash
# Round 6: does the default bench's short warm-up (5 steps, ~11 ms) leave the device below its settled clock?
# (tools/r06_warmup.sh TAG): the main line alone with warm-up 5 / 300 / 5, steps 20 / 20 / 200
mkdir -p gpurun_out
export TMPDIR=/tmp
F="--no-cpu-baseline --no-alt --no-train --north-star-cfg 0 --roofline-cfg 0 --batch-cfg 0 --no-probe"
for wk in "5 20" "300 20" "5 200" "5 20"; do
  set -- $1 $wk
  timeout -k 10 300 python bench.py $F --warmup $2 --steps $3 >> gpurun_out/$1_warmup.jsonl 2>> gpurun_out/$1_warmup.err || { tail -20 gpurun_out/$1_warmup.err; exit 1; }
done
python - "$1" <<'P'
import json, sys
for l in open(f"gpurun_out/{sys.argv[1]}_warmup.jsonl"):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l)
        print(d["warmup"], d["steps"], d["value"], d["ms_per_step"], d.get("stages_ms"))
P
