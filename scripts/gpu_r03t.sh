#!/bin/bash
# GPU box: frames in flight, 8K (18 / 20 / 22) and C5 (16 / 20), HBM-resident
# value, 5 timed steps each, no PCIe / CPU legs.
set -o pipefail
TAG=${1:-r03t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in 8k:20 8k:18 8k:22 c5:16 c5:20 8k:16; do
  wl=${spec%%:*}; c=${spec##*:}
  timeout -k 10 300 python -u bench.py --workload $wl --concurrency $c --no-cpu-baseline --no-pcie > $OUT/bench_${wl}_c$c.json 2> $OUT/bench_${wl}_c$c.err || { echo "bench $spec failed"; tail -20 $OUT/bench_${wl}_c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $OUT/bench_${wl}_c$c.json $spec
done
