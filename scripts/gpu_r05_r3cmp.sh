# single-frame latency: the other build (_rXtree, git worktree of d9d92bd) against this one, alternating
set -o pipefail
T=${1:-r05c3}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
(cd ${2:-_r3tree} && timeout -k 10 300 python3 -u scripts/probe_perf.py 512 4k) > gpurun_out/$T/r3_$r.txt 2>&1 || { tail -20 gpurun_out/$T/r3_$r.txt; exit 1; }
echo "other build, run $r"; grep -v "^  \|amdgpu.ids" gpurun_out/$T/r3_$r.txt
grep "^  enc\|^  dec" gpurun_out/$T/r3_$r.txt | python3 -c "
import sys, ast
for l in sys.stdin:
    k, d = l.strip().split(' ', 1); d = ast.literal_eval(d); print('   ', k, 't1_ms', d['t1_ms'])"
timeout -k 10 300 python3 -u scripts/probe_perf.py 512 4k > gpurun_out/$T/r5_$r.txt 2>&1 || { tail -20 gpurun_out/$T/r5_$r.txt; exit 1; }
echo "round-5 build, run $r"; grep -v "^  \|amdgpu.ids" gpurun_out/$T/r5_$r.txt
grep "^  enc\|^  dec" gpurun_out/$T/r5_$r.txt | python3 -c "
import sys, ast
for l in sys.stdin:
    k, d = l.strip().split(' ', 1); d = ast.literal_eval(d); print('   ', k, 't1_ms', d['t1_ms'])"
done
