# A/B of the T1 decoder's workgroup shape (GRKGPU_T1_DEC_WG 1 | 4):
# bench lines of both, then the GPU suite under the 4-wavefront shape
set -o pipefail
T=${1:-r05d}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for wg in 1 4 1 4; do
GRKGPU_T1_DEC_WG=$wg timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench_wg$wg.json 2> gpurun_out/$T/bench_wg$wg.err || { tail -30 gpurun_out/$T/bench_wg$wg.err; exit 1; }
python3 - gpurun_out/$T/bench_wg$wg.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lf = d["t1"]["lone_frame"]
print(sys.argv[1], "value", d["value"], "dec_t1_ms", lf["dec_t1_ms"], "enc_t1_ms", lf["enc_t1_ms"], "batch_msym", d["t1"]["batch_enc_dec_msym_per_s"])
PY
done
GRKGPU_T1_DEC_WG=4 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_wg4.txt 2>&1; tail -3 gpurun_out/$T/pytest_wg4.txt
