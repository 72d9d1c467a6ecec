#!/bin/bash
# GPU box: full parity suite, lone-frame latency of every BASELINE config,
# and the C5 / C4 bench workloads.  Usage: bash scripts/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 400 python -u scripts/probe_perf.py 512 4k 8k 16k > $OUT/probe_all.txt 2>&1 || { echo "probe failed"; tail $OUT/probe_all.txt; exit 1; }
grep Mpix $OUT/probe_all.txt
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-pcie > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "c5 bench failed"; tail $OUT/bench_c5.err; exit 1; }
tail -1 $OUT/bench_c5.json | cut -c1-300
