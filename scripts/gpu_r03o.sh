#!/bin/bash
# GPU box: T1 A/B (A = lib_ab/ = HEAD, B = lib/ = working tree; 3 alternating
# rounds of scripts/t1_ab.py), then the 8K and C5 bench lines on B.
set -o pipefail
TAG=${1:-r03o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/gpu_ab.sh $TAG/ab 3 || exit 1
for wl in 8k c5; do
  timeout -k 10 400 python -u bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo "bench $wl failed"; tail -30 $OUT/bench_$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['pcie_inclusive']['value'], d['roofline']['frac'])" $OUT/bench_$wl.json
done
