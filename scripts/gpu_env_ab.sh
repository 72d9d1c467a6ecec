# A/B of an environment switch on the 8K bench: bash scripts/gpu_env_ab.sh TAG VAR v1 v2 ...
# (two alternating rounds over the values), then the encode / T1 GPU tests under the last value
set -o pipefail
T=$1; V=$2; shift 2
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
for v in "$@"; do
env $V=$v timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench_${v}_$r.json 2> gpurun_out/$T/bench_${v}_$r.err || { tail -30 gpurun_out/$T/bench_${v}_$r.err; exit 1; }
python3 - gpurun_out/$T/bench_${v}_$r.json "$V=$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lf = d["t1"]["lone_frame"]
print(sys.argv[2], "value", d["value"], "dec_t1_ms", lf["dec_t1_ms"], "enc_t1_ms", lf["enc_t1_ms"], "batch_msym", d["t1"]["batch_enc_dec_msym_per_s"])
PY
done
done
for v in "$@"; do last=$v; done
env $V=$last timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1; tail -2 gpurun_out/$T/pytest.txt
