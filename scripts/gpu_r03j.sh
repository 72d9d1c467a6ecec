#!/bin/bash
# GPU box: multiply issue-rate probe, forward-DWT span A/B (A = lib_ab built
# with -DGRK_FIXMUL64, B = lib/ with the 24-bit fixmul13), then the GPU suite.
# Usage: bash scripts/gpu_r03j.sh TAG
set -o pipefail
TAG=${1:-r03j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 60 ./scripts/mulrate > $OUT/mulrate.txt 2>&1 || { echo "mulrate failed"; cat $OUT/mulrate.txt; exit 1; }
cat $OUT/mulrate.txt
AB=$PWD/grokimagecompression_amd/lib_ab/libgrk_mi355x.so
for round in 1 2; do
  GRKGPU_LIB=$AB timeout -k 10 200 python -u scripts/dwt_span_ab.py "" > $OUT/A_$round.json 2> $OUT/A_$round.err || { echo "A failed"; tail $OUT/A_$round.err; exit 1; }
  echo "A$round $(cat $OUT/A_$round.json)"
  timeout -k 10 200 python -u scripts/dwt_span_ab.py "" > $OUT/B_$round.json 2> $OUT/B_$round.err || { echo "B failed"; tail $OUT/B_$round.err; exit 1; }
  echo "B$round $(cat $OUT/B_$round.json)"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
