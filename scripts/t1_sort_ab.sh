#!/bin/bash
# GPU box: A/B of the T1 decoder's lane assignment on the lone 8K frame --
# block order (t1_dec_sort 0 / 1) and blocks per wavefront (t1_dec_bpw) --
# alternating, ROUNDS times.  Usage: bash scripts/t1_sort_ab.sh TAG [spec ...]
# (spec: space-free option lists like "t1_dec_sort=1,t1_dec_bpw=16"; "-" = defaults)
set -o pipefail
TAG=${1:-sortab}
shift
SPECS=${@:-"- t1_dec_sort=1"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $SPECS; do
    args=$(echo "$v" | tr ',' ' '); [ "$v" = "-" ] && args=""
    timeout -k 10 200 python -u scripts/probe_perf.py 8k $args > $OUT/probe_${v}_$round.txt 2>&1 || { echo "probe $v failed"; tail $OUT/probe_${v}_$round.txt; exit 1; }
    echo "$v r$round $(grep -o "dec {[^}]*'t1_ms': [0-9.]*" $OUT/probe_${v}_$round.txt | grep -o "t1_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
