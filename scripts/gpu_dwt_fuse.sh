#!/bin/bash
# GPU box: parity suite, then per-level DWT kernel times for the fused
# DC shift + MCT level 0 at several window heights.  Usage: bash scripts/gpu_dwt_fuse.sh TAG
set -o pipefail
TAG=${1:-dwtfuse}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for spec in "GRKGPU_DWT_FUSE=0" "GRKGPU_DWT_FUSE=1" "GRKGPU_DWT_FUSE=1,GRKGPU_DWT_TH=8" "GRKGPU_DWT_FUSE=1,GRKGPU_DWT_TH=16" "GRKGPU_DWT_BIGMIN=30000000" "GRKGPU_DWT_TH=16"; do
  n=$(echo $spec | tr ',=' '__')
  bash scripts/dwt_levels.sh $TAG/$n $(echo $spec | tr ',' ' ') > /dev/null || { echo "levels $spec failed"; exit 1; }
  echo "== $spec"; grep -E "dwt_fwd|dcshift" $OUT/$n/levels.txt
done
