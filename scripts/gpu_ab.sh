#!/bin/bash
# GPU box: A/B of two library builds on one box -- A = lib_ab/ (the
# reference build), B = lib/ (the change) -- alternating runs of
# scripts/t1_ab.py (lone-frame T1 medians, 16-context batch throughput).
# Usage: bash scripts/gpu_ab.sh TAG [rounds]
set -o pipefail
TAG=${1:-ab}
N=${2:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=20
AB=$PWD/grokimagecompression_amd/lib_ab/libgrk_mi355x.so
for round in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then export GRKGPU_LIB=$AB; else unset GRKGPU_LIB; fi
    timeout -k 10 300 python -u scripts/t1_ab.py > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err || { echo "run $v failed"; tail $OUT/${v}_$round.err; exit 1; }
    echo "$v$round $(cat $OUT/${v}_$round.json)"
  done
done
