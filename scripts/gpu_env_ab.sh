#!/bin/bash
# GPU box: parity suite, then lone-frame stage times (probe_perf 8k) and the
# default bench line for each env setting, two alternating rounds.
# Usage: bash scripts/gpu_env_ab.sh TAG "ENV=V[,ENV2=V2]" "ENV=V" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
  tail -1 $OUT/pytest_gpu.txt
fi
for round in 1 2; do
  i=0
  for spec in "$@"; do
    i=$((i+1))
    ( export $(echo $spec | tr ',' ' ')
      timeout -k 10 200 python -u scripts/probe_perf.py 8k > $OUT/probe_${i}_$round.txt 2>&1 || exit 1
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie > $OUT/bench_${i}_$round.json 2> $OUT/bench_${i}_$round.err || exit 1
    ) || { echo "run $spec failed"; tail -5 $OUT/probe_${i}_$round.txt $OUT/bench_${i}_$round.err; exit 1; }
    echo "$spec r$round $(grep -o '"value": [0-9.]*' $OUT/bench_${i}_$round.json) lone: $(grep -o "Mpix/s=[0-9.]*" $OUT/probe_${i}_$round.txt | tr '\n' ' ') enc_t1: $(grep -o "enc {[^}]*'t1_ms': [0-9.]*" $OUT/probe_${i}_$round.txt | grep -o "t1_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
