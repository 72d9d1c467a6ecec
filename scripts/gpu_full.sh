#!/bin/bash
# GPU box: the whole -m gpu suite, then the default bench line.  Usage: bash scripts/gpu_full.sh TAG
set -o pipefail
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'])"
