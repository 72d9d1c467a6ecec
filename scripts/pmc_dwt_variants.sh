#!/bin/bash
# PMC passes over scripts/dwt_bench.py for DWT kernel variants.
# Usage: bash scripts/pmc_dwt_variants.sh TAG "ENV=..,ENV=.." ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
P2="FETCH_SIZE TCC_HIT_sum"
P3="WRITE_SIZE TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum"
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=$(echo $spec | tr ',' ' ')
  j=0; mkdir -p $OUT/v$i
  for P in "$P1" "$P2" "$P3"; do
    j=$((j+1))
    (export $envs; timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/v$i/p$j -o run -- python3 scripts/dwt_bench.py > $OUT/v$i/p$j.log 2>&1) || { echo "pmc v$i p$j failed"; tail -5 $OUT/v$i/p$j.log; exit 1; }
  done
  echo "v$i: $spec"
done
