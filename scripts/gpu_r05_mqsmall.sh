# single-wavefront MQ workgroups for lone / small encodes: 512^2 kernel times,
# lone-call latencies, the GPU parity suite and the default bench line
set -o pipefail
T=${1:-r05m1}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run -- python3 -u scripts/probe_perf.py 512 > gpurun_out/$T/p512.txt 2>&1 || { tail -20 gpurun_out/$T/p512.txt; exit 1; }
python3 scripts/prof_summary.py gpurun_out/$T/prof gpurun_out/$T/ks.csv > /dev/null && head -8 gpurun_out/$T/ks.csv
timeout -k 10 300 python3 -u scripts/probe_perf.py 512 4k 8k > gpurun_out/$T/probe.txt 2>&1 || { tail -20 gpurun_out/$T/probe.txt; exit 1; }
cat gpurun_out/$T/probe.txt | tail -30
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/$T/gpu_tests.txt
timeout -k 10 300 python3 -u bench.py > gpurun_out/$T/bench.txt 2>&1 || { tail -20 gpurun_out/$T/bench.txt; exit 1; }
tail -1 gpurun_out/$T/bench.txt
