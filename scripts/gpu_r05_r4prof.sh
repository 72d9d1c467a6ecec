# per-kernel times of the 512^2 config: the round-4 build (_r4tree) and this one
set -o pipefail
T=${1:-r05p4}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
(cd _r4tree && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/$T/prof4 -o run -- python3 -u scripts/probe_perf.py 512) > gpurun_out/$T/p4.txt 2>&1 || { tail -20 gpurun_out/$T/p4.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof5 -o run -- python3 -u scripts/probe_perf.py 512 > gpurun_out/$T/p5.txt 2>&1 || { tail -20 gpurun_out/$T/p5.txt; exit 1; }
for v in 4 5; do python3 scripts/prof_summary.py gpurun_out/$T/prof$v gpurun_out/$T/ks$v.csv > /dev/null && echo "== round $v" && head -8 gpurun_out/$T/ks$v.csv; done
