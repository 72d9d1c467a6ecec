# lone-call latency: the model's conditional row reads (GRKGPU_T1_MODEL_COND) and a
# single-wavefront, uncapped decoder for lone / small launches (GRKGPU_T1_DEC_LONE_WG1)
set -o pipefail
T=${1:-r05l2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for combo in "1 0" "0 0" "1 1" "0 1" "1 0" "0 1"; do
set -- $combo
GRKGPU_T1_MODEL_COND=$1 GRKGPU_T1_DEC_LONE_WG1=$2 timeout -k 10 300 python3 -u scripts/probe_perf.py 512 4k 8k > gpurun_out/$T/p_$1_$2.txt 2>&1 || { tail -20 gpurun_out/$T/p_$1_$2.txt; exit 1; }
echo "model_cond=$1 dec_lone_wg1=$2"; grep -v "^  " gpurun_out/$T/p_$1_$2.txt | grep -v amdgpu.ids
grep "^  enc\|^  dec" gpurun_out/$T/p_$1_$2.txt | python3 -c "
import sys, ast
for l in sys.stdin:
    k, d = l.strip().split(' ', 1); d = ast.literal_eval(d); print('   ', k, 't1_ms', d['t1_ms'])"
done
