#!/bin/bash
# round 3 measurement set: rocprofv3 kernel stats of the default bench (3
# steps), then the HBM traffic passes (FETCH_SIZE, WRITE_SIZE) of a 1-frame
# bench -> gpurun_out/TAG/{kernel_stats.csv, pmc/pmc_summary.json}
set -o pipefail
TAG=${1:-r03prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=20
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
head -16 $OUT/kernel_stats.csv
bash scripts/pmc_bench.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
tail -3 $OUT/pmc.log
