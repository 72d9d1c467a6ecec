#!/bin/bash
# GPU box: frames in flight for the HBM-resident 8K value (16 / 20 / 24 /
# 16 again), 5 timed steps each, no PCIe / CPU legs.
set -o pipefail
TAG=${1:-r03s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in 16 20 24 16; do
  timeout -k 10 300 python -u bench.py --concurrency $c --no-cpu-baseline --no-pcie > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { echo "bench c$c failed"; tail -20 $OUT/bench_c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $OUT/bench_c$c.json $c
done
