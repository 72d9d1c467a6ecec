#!/bin/bash
# GPU box: the -m gpu suite.  Usage: bash scripts/gpu_pytest.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-pytest}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
