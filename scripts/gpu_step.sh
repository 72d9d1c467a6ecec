#!/bin/bash
# GPU box helper: run one named step with its own time limit, output under
# gpurun_out/<tag>/; stops the chain on the first failure.
#   bash scripts/gpu_step.sh TAG pytest "<-k expr>"      -m gpu tests (subset)
#   bash scripts/gpu_step.sh TAG prof "<python args>"    rocprofv3 kernel stats of a python command
#   bash scripts/gpu_step.sh TAG run "<python args>"     plain python command
set -o pipefail
TAG=$1; KIND=$2; ARGS=$3; LIMIT=${4:-600}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
case $KIND in
  pytest)
    timeout -k 10 $LIMIT python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${ARGS:+-k "$ARGS"} > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
    tail -2 $OUT/pytest_gpu.txt ;;
  prof)
    timeout -k 10 $LIMIT rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u $ARGS > $OUT/out.txt 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
    python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
    cat $OUT/out.txt; head -30 $OUT/kernel_stats.csv | cut -c1-160 ;;
  run)
    timeout -k 10 $LIMIT python3 -u $ARGS > $OUT/out.txt 2>&1 || { echo "run failed"; tail -30 $OUT/out.txt; exit 1; }
    tail -30 $OUT/out.txt ;;
esac
