#!/bin/bash
# GPU box: timed steps K of the HBM-resident 8K value (5 / 10 / 20 / 5):
# how much of a short run is pipeline fill and drain.
set -o pipefail
TAG=${1:-r03v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for k in 5 10 20 5; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps $k --no-cpu-baseline --no-pcie > $OUT/bench_k${k}_$i.json 2> $OUT/bench_k${k}_$i.err || { echo "bench k$k failed"; tail -20 $OUT/bench_k${k}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $OUT/bench_k${k}_$i.json $k
done
