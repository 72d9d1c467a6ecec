#!/bin/bash
# GPU box: DWT plan variants (f01_rows 8, small_rows 24; both measured slower
# and removed again, profiles/r03_dwt_valu_ab.txt) -- span A/B and the
# per-launch times, then their parity tests.
set -o pipefail
TAG=${1:-r03k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u scripts/dwt_span_ab.py "" "f01_rows=8" "small_rows=24" "f01_rows=8,small_rows=24" "f01_rows=6" > $OUT/span.json 2> $OUT/span.err || { echo "span failed"; tail $OUT/span.err; exit 1; }
cat $OUT/span.json
timeout -k 10 300 python -u scripts/dwt_launch_probe.py "" "f01_rows=8,small_rows=24" > $OUT/launch.txt 2>&1 || { echo "probe failed"; tail $OUT/launch.txt; exit 1; }
grep -v amdgpu.ids $OUT/launch.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small_rows or fused01" > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
