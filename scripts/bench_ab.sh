#!/bin/bash
# GPU box: the default bench line (16 frames in flight) under plan options,
# alternating, ROUNDS times.  Usage: bash scripts/bench_ab.sh TAG WORKLOAD [spec ...]
# (spec: "k=v,k=v"; "-" = defaults)
set -o pipefail
TAG=${1:-benchab}
WL=${2:-8k}
shift 2
SPECS=${@:-"- t1_dec_sort=1"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $SPECS; do
    opt=$v; [ "$v" = "-" ] && opt=""
    timeout -k 10 300 python -u bench.py --workload $WL --no-cpu-baseline --no-pcie ${opt:+--opt $opt} > $OUT/bench_${v}_$round.json 2> $OUT/bench_${v}_$round.err || { echo "bench $v failed"; tail $OUT/bench_${v}_$round.err; exit 1; }
    echo "$v r$round $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$round.json)"
  done
done
