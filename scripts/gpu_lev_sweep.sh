#!/bin/bash
# GPU box: per-level DWT kernel times under several env settings (no tests).
# Usage: bash scripts/gpu_lev_sweep.sh TAG "ENV=V[,ENV2=V2]" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
  n=$(echo $spec | tr ',=' '__')
  bash scripts/dwt_levels.sh $TAG/$n $(echo $spec | tr ',' ' ') > /dev/null || { echo "levels $spec failed"; exit 1; }
  echo "== $spec"; grep -E "dwt_fwd.*true|fwd01" $OUT/$n/levels.txt
done
