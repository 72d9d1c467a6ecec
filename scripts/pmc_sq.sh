#!/bin/bash
# SQ instruction / wait counters for the bench kernels, one pass per env setting.
# Usage: bash scripts/pmc_sq.sh TAG "ENV=..." ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
i=0
for E in "$@"; do
  i=$((i+1))
  export $E
  GPU_MAX_HW_QUEUES=16 timeout -s KILL 180 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/run$i -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --concurrency 1 > $OUT/run$i.log 2>&1 || { echo "pmc run $i failed"; tail -5 $OUT/run$i.log; exit 1; }
  unset ${E%%=*}
  echo "run$i: $E"
done
