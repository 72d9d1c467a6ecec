#!/bin/bash
# round 3: GPU suite + C4 bench + C4 shard probe, then the T1 SQ counters
set -o pipefail
TAG=${1:-r03i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_suite.sh $TAG c4 || exit 1
timeout -k 10 300 python -u scripts/c4_probe.py > $OUT/c4_probe.txt 2>&1 || { echo "c4 probe failed"; tail -20 $OUT/c4_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/c4_probe.txt | cut -c1-300
bash scripts/gpu_sq.sh $TAG/sq
