#!/bin/bash
# GPU-box routine: parity tests, HBM-traffic PMC passes, bench line, rocprofv3
# kernel stats of the bench.  Usage (repo root, on the box): bash scripts/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
bash scripts/pmc_bench.sh $TAG/pmc > /dev/null || { echo "pmc failed"; exit 1; }
cp $OUT/pmc/pmc_summary.json profiles/dwt_pmc_latest.json
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --concurrency 1 > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -30 $OUT/prof.err; exit 1; }
python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
head -16 $OUT/kernel_stats.csv
