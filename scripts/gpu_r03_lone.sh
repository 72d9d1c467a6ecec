#!/bin/bash
# lone-frame kernel stats (one frame at a time, nothing else in flight):
# rocprofv3 over scripts/probe_perf.py 8k -> gpurun_out/TAG/kernel_stats.csv
set -o pipefail
TAG=${1:-r03lone}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u scripts/probe_perf.py 8k > $OUT/probe.txt 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
head -24 $OUT/kernel_stats.csv
grep -v amdgpu.ids $OUT/probe.txt | tail -8
