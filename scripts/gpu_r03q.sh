#!/bin/bash
# GPU box, round-3 closing profiles: lone-frame kernel stats, SQ counters of
# the T1 kernels, HBM traffic PMC passes, kernel stats of the 16-frame bench.
set -o pipefail
TAG=${1:-r03q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_r03_lone.sh $TAG/lone > $OUT/lone.log 2>&1 || { echo "lone failed"; tail $OUT/lone.log; exit 1; }
head -14 $OUT/lone/kernel_stats.csv
bash scripts/gpu_sq.sh $TAG/sq > $OUT/sq.log 2>&1 || { echo "sq failed"; tail $OUT/sq.log; exit 1; }
cat $OUT/sq/sq.txt
bash scripts/pmc_bench.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail $OUT/pmc.log; exit 1; }
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-pcie --steps 3 --warmup 1 > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof bench failed"; tail -20 $OUT/prof.err; exit 1; }
python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats_batch.csv > /dev/null
head -12 $OUT/kernel_stats_batch.csv
