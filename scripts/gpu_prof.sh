#!/bin/bash
# GPU box: rocprofv3 kernel stats of one bench configuration.  Usage: bash scripts/gpu_prof.sh TAG [bench args]
set -o pipefail
TAG=${1:-prof}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-pcie "$@" > $OUT/bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
head -14 $OUT/kernel_stats.csv
