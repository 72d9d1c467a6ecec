#!/bin/bash
# SQ counters of the T1 kernels for one 8K 9/7 encode + decode: two rocprofv3
# --pmc passes (instruction mix and waits; VALU lane activity), each its own run.
# Usage: bash scripts/gpu_sq.sh TAG -> gpurun_out/TAG/sq.txt
set -o pipefail
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 -u scripts/t1_sq_probe.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/sq_pass_table.py $OUT/p1 $OUT/p2 > $OUT/sq.txt && cat $OUT/sq.txt
