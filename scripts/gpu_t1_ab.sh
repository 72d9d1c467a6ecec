#!/bin/bash
# GPU box: T1 parity tests, then an A/B of the in-tree library vs lib_ab/
# (lone-frame stage times + bench line, alternating).  Usage: bash scripts/gpu_t1_ab.sh TAG
set -o pipefail
TAG=${1:-t1ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
bash scripts/gpu_ab_lib.sh $TAG/ab
