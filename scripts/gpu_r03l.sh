#!/bin/bash
# GPU box: T1 A/B (A = lib_ab/ = HEAD, B = lib/ = working tree), 3 alternating
# rounds of scripts/t1_ab.py, then the GPU suite on B.
set -o pipefail
TAG=${1:-r03l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/gpu_ab.sh $TAG/ab 3 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
