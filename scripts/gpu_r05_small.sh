# per-kernel times of the 512^2 config (BASELINE configs[0]) under rocprofv3
set -o pipefail
T=${1:-r05s}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run -- python3 -u scripts/probe_perf.py 512 > gpurun_out/$T/probe.txt 2> gpurun_out/$T/prof.err || { tail -20 gpurun_out/$T/prof.err; exit 1; }
grep -v "^  " gpurun_out/$T/probe.txt
python3 scripts/prof_summary.py gpurun_out/$T/prof gpurun_out/$T/kernel_stats.csv > /dev/null && head -14 gpurun_out/$T/kernel_stats.csv
