#!/bin/bash
# GPU box: SQ counters (two --pmc passes) of the lone 8K frame's kernels for
# each env setting.  Usage: bash scripts/gpu_sq_env.sh TAG "ENV=V" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
i=0
for spec in "$@"; do
  i=$((i+1))
  j=0
  for P in "$P1" "$P2"; do
    j=$((j+1))
    ( export $(echo $spec | tr ',' ' '); timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/e${i}_sq$j -o run -- python3 -u scripts/probe_perf.py 8k > $OUT/e${i}_sq$j.log 2>&1 ) || { echo "pmc $spec pass $j failed"; tail -5 $OUT/e${i}_sq$j.log; exit 1; }
  done
  echo "$spec done"
done
