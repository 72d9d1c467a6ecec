#!/bin/bash
# GPU box: rocprofv3 kernel stats of a short bench run (the roofline check
# against the bench line's own launch times), then the HBM counter passes of
# a 1-step bench (scripts/pmc_bench.sh) for roofline.traffic.
set -o pipefail
TAG=${1:-r05p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-pcie --steps 2 --warmup 1 --concurrency 2 > $OUT/bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
python3 scripts/roofline_check.py $OUT/prof $OUT/bench.json | tee $OUT/roofline_check.txt
bash scripts/pmc_bench.sh ${TAG}_pmc
