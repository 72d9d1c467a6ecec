#!/bin/bash
# Kernel trace of scripts/dwt_bench.py (8K 12-bit RGB, 9/7 + 5/3 enc + dec) ->
# per-launch DWT durations (scripts/dwt_levels.py).  Usage: bash scripts/dwt_levels.sh TAG [ENV=V ...]
set -o pipefail
TAG=${1:-dwtlev}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 -u scripts/dwt_bench.py > $OUT/bench.txt 2>&1 || { echo "trace failed"; tail -5 $OUT/bench.txt; exit 1; }
grep -v amdgpu.ids $OUT/bench.txt
python3 scripts/dwt_levels.py $OUT/trace | tee $OUT/levels.txt
