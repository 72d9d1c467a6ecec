#!/bin/bash
# GPU box: A/B of plan options on the lone 8K frame (probe_perf: T1 decode
# times) AND on the 16-frame batch bench line, alternating, ROUNDS times.
# Usage: bash scripts/t1_bpw_ab.sh TAG [spec ...]   (spec: "k=v,k=v"; "-" = defaults)
set -o pipefail
TAG=${1:-bpwab}
shift
SPECS=${@:-"- t1_dec_bpw=16"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for round in $(seq 1 ${ROUNDS:-1}); do
  for v in $SPECS; do
    args=$(echo "$v" | tr ',' ' '); [ "$v" = "-" ] && args=""
    opt=$v; [ "$v" = "-" ] && opt=""
    timeout -k 10 200 python -u scripts/probe_perf.py 8k $args > $OUT/probe_${v}_$round.txt 2>&1 || { echo "probe $v failed"; tail $OUT/probe_${v}_$round.txt; exit 1; }
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie ${opt:+--opt $opt} > $OUT/bench_${v}_$round.json 2> $OUT/bench_${v}_$round.err || { echo "bench $v failed"; tail $OUT/bench_${v}_$round.err; exit 1; }
    echo "$v r$round $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$round.json) dec $(grep -o "dec {[^}]*'t1_ms': [0-9.]*" $OUT/probe_${v}_$round.txt | grep -o "t1_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
