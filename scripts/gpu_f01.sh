#!/bin/bash
# GPU box: parity suite, then per-level DWT kernel times with the fused
# 9/7 levels 0+1 (default) and without (GRKGPU_DWT_F01=0).  Usage: bash scripts/gpu_f01.sh TAG
set -o pipefail
TAG=${1:-f01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for spec in ${SPECS:-"GRKGPU_DWT_F01=4" "GRKGPU_DWT_F01=0"}; do
  n=$(echo $spec | tr ',=' '__')
  bash scripts/dwt_levels.sh $TAG/$n $(echo $spec | tr ',' ' ') > /dev/null || { echo "levels $spec failed"; exit 1; }
  echo "== $spec"; grep -E "dwt_fwd|dcshift" $OUT/$n/levels.txt
done
