#!/bin/bash
# round 3: GPU suite + 8K bench, then the frames-in-flight sweep of the H2D-inclusive value
set -o pipefail
TAG=${1:-r03g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_suite.sh $TAG 8k || exit 1
for c in 16 20; do
  timeout -k 10 300 python -u bench.py --concurrency $c --no-cpu-baseline > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { echo "bench c$c failed"; tail -20 $OUT/bench_c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['hbm_resident']['value'])" $OUT/bench_c$c.json
done
