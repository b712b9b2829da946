#!/bin/bash
# Round 6: warp parity + A/B timing, then the profile set (tools/r06_warp2.sh TAG)
set -o pipefail
bash tools/r06_warp.sh $1 || exit $?
timeout -k 10 900 bash tools/profile_gpu.sh $1 2 > gpurun_out/$1_profile.log 2>&1 || { tail -20 gpurun_out/$1_profile.log; exit 1; }
tail -3 gpurun_out/$1_profile.log
