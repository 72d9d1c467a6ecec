#!/bin/bash
# GPU box: selected GPU tests (-k EXPR) then one bench line.  Usage: bash scripts/gpu_quick.sh TAG "pytest -k expr" [bench args]
set -o pipefail
TAG=${1:-quick}
K=${2:-}
shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
timeout -k 10 400 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
