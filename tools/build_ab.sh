#!/bin/bash
# Build libmvbev.so from a git revision into mvdet_amd/lib/exp/libmvbev_<name>.so (A/B runs with
# tools/kbench.py --libs).  Usage: bash tools/build_ab.sh <rev> <name> [EXTRA flags]
set -e
REV=$1; NAME=$2; EXTRA=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive "$REV" mvdet_amd/csrc include | tar -x -C "$T"
make -C "$T/mvdet_amd/csrc" -j8 OUT="$R/mvdet_amd/lib/exp/libmvbev_$NAME.so" OBJDIR="$T/obj" EXTRA="$EXTRA" >/dev/null
rm -rf "$T"
echo "$R/mvdet_amd/lib/exp/libmvbev_$NAME.so"
