# forward 9/7 tail: levels 3 + 4 as one k_dwt_fwd01 launch (GRKGPU_F01_TAIL=1) vs apart, alternating
set -o pipefail
T=${1:-r05t}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2 3; do
for v in 0 1; do
GRKGPU_F01_TAIL=$v timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/$T/b_${v}_$r.json 2> gpurun_out/$T/b_${v}_$r.err || { tail -30 gpurun_out/$T/b_${v}_$r.err; exit 1; }
python3 - gpurun_out/$T/b_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("tail", sys.argv[2], "span %.1f frac %.4f" % (r["span_us"], r["frac"]), " ".join("%s L%d+%d %.1f" % (x["kernel"], x["levels"][0], len(x["levels"]), x["us"]) for x in r["launches"]))
PY
done
done
GRKGPU_F01_TAIL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dwt or encode" > gpurun_out/$T/pytest.txt 2>&1; tail -1 gpurun_out/$T/pytest.txt
