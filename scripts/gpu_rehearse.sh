#!/bin/bash
# GPU box: what the driver runs at round end -- smoke(), then the default
# bench line -- plus a rocprofv3 --stats of a short bench.  Usage: bash scripts/gpu_rehearse.sh TAG
set -o pipefail
TAG=${1:-rehearse}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-200
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-pcie --steps 3 --warmup 1 > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
head -12 $OUT/kernel_stats.csv
