#!/bin/bash
# GPU box: A/B of decoder block order (t1_dec_sort 0 / 1) on the lone 8K
# frame, alternating, ROUNDS times.  Usage: bash scripts/t1_sort_ab.sh TAG
set -o pipefail
TAG=${1:-sortab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in 0 1; do
    timeout -k 10 200 python -u scripts/probe_perf.py 8k t1_dec_sort=$v > $OUT/probe_${v}_$round.txt 2>&1 || { echo "probe $v failed"; tail $OUT/probe_${v}_$round.txt; exit 1; }
    echo "sort=$v r$round $(grep -o "dec {[^}]*'t1_ms': [0-9.]*" $OUT/probe_${v}_$round.txt | grep -o "t1_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
