# the other bench lines: C5 cinema (twice), C4 tile shards, and the 8K frame
# batch with two ranks sharing the one GPU (per-rank host Tier-2 for DESIGN 6)
set -o pipefail
T=${1:-r05l}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 10 --warmup 2 > gpurun_out/$T/bench_c5_$r.json 2> gpurun_out/$T/bench_c5_$r.err || { tail -30 gpurun_out/$T/bench_c5_$r.err; exit 1; }
python3 - gpurun_out/$T/bench_c5_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d.get("stage_ms", {})
print(sys.argv[1], "value", d["value"], {k: (v.get("t1_ms"), v.get("host_t2_ms"), v.get("rate_ms")) for k, v in st.items()})
PY
done
timeout -k 10 400 python3 -u bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/$T/bench_c4.json 2> gpurun_out/$T/bench_c4.err || { tail -30 gpurun_out/$T/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4', d['value'])" gpurun_out/$T/bench_c4.json
timeout -k 10 500 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/bench_g2.json 2> gpurun_out/$T/bench_g2.err || { tail -30 gpurun_out/$T/bench_g2.err; exit 1; }
python3 - gpurun_out/$T/bench_g2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d.get("stage_ms", {})
print("gpus2 value", d["value"], "n_gpus", d["n_gpus"], "ms_per_step", d["ms_per_step"], {k: (v.get("t1_ms"), v.get("host_t2_ms")) for k, v in st.items()})
PY
bash scripts/gpu_sq.sh ${T}_sq || exit 1
