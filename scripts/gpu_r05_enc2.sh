# conditional row reads in the model kernel: GPU suite, two bench lines, then
# rocprof stats + roofline check + HBM counter passes (scripts/gpu_r05_prof.sh)
set -o pipefail
T=${1:-r05g}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_full.txt 2>&1 || { tail -40 gpurun_out/$T/pytest_full.txt; exit 1; }
tail -1 gpurun_out/$T/pytest_full.txt
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench_$r.json 2> gpurun_out/$T/bench_$r.err || { tail -30 gpurun_out/$T/bench_$r.err; exit 1; }
python3 - gpurun_out/$T/bench_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lf = d["t1"]["lone_frame"]
print(sys.argv[1], "value", d["value"], "frac", d["roofline"]["frac"], "inv", d["roofline"]["inverse"]["frac"], "dec_t1_ms", lf["dec_t1_ms"], "enc_t1_ms", lf["enc_t1_ms"])
PY
done
bash scripts/gpu_r05_prof.sh ${T}p > /dev/null || exit 1
cat gpurun_out/${T}p/roofline_check.txt
python3 - gpurun_out/${T}p_pmc/pmc_summary.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
for k, v in b["kernels"].items():
    if "t1" in k or "mq" in k:
        print(k, [(e["dispatches"], round(e["read_bytes"] / 1e6), round(e["write_bytes"] / 1e6)) for e in v])
PY
