#!/bin/bash
# GPU box: smoke(), the whole -m gpu suite, then one bench line per workload
# given (e.g. "8k" "c5").  Usage: bash scripts/gpu_suite.sh TAG [workload ...]
set -o pipefail
TAG=${1:-suite}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for wl in "$@"; do
  timeout -k 10 400 python -u bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo "bench $wl failed"; tail -30 $OUT/bench_$wl.err; exit 1; }
  cat $OUT/bench_$wl.json
done
