#!/bin/bash
# HBM traffic of the bench's kernels: one rocprofv3 --pmc pass per counter
# (FETCH_SIZE, WRITE_SIZE), each over a 1-step bench run; then summarise into
# profiles/<tag>_pmc.json (read by bench.py for roofline.traffic).
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  GPU_MAX_HW_QUEUES=16 timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$C -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --concurrency 1 > $OUT/$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
python3 scripts/pmc_summary.py $OUT $OUT/pmc_summary.json && cat $OUT/pmc_summary.json
