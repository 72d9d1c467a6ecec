#!/bin/bash
# GPU box: A/B of two library builds (default lib/ vs lib_ab/): lone-frame
# stage times (probe_perf 8k) and the default bench line, alternating.
# Usage: bash scripts/gpu_ab_lib.sh TAG
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
AB=$PWD/grokimagecompression_amd/lib_ab/libgrk_mi355x.so
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in A B; do
    if [ $v = B ]; then export GRKGPU_LIB=$AB; else unset GRKGPU_LIB; fi
    timeout -k 10 200 python -u scripts/probe_perf.py 8k > $OUT/probe_${v}_$round.txt 2>&1 || { echo "probe $v failed"; tail $OUT/probe_${v}_$round.txt; exit 1; }
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie > $OUT/bench_${v}_$round.json 2> $OUT/bench_${v}_$round.err || { echo "bench $v failed"; tail $OUT/bench_${v}_$round.err; exit 1; }
    echo "$v$round $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$round.json) $(grep -o "dec {[^}]*'t1_ms': [0-9.]*" $OUT/probe_${v}_$round.txt | grep -o "t1_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
