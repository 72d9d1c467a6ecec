# DWT occupancy A/B: k_dwt_inv01 held to 6 (9/7) / 4 (5/3) wavefronts per SIMD
# (GRKGPU_INV01_WPE=6) and the 5/3 DC shift + RCT level 0 to 5 (GRKGPU_MCT3_WPE=5), alternating
set -o pipefail
T=${1:-r05o}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2 3; do
for v in 0 1; do
if [ $v = 1 ]; then export GRKGPU_INV01_WPE=6 GRKGPU_MCT3_WPE=5; else unset GRKGPU_INV01_WPE GRKGPU_MCT3_WPE; fi
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/$T/b_${v}_$r.json 2> gpurun_out/$T/b_${v}_$r.err || { tail -30 gpurun_out/$T/b_${v}_$r.err; exit 1; }
python3 - gpurun_out/$T/b_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; r53 = r["r53"]
print("variant", sys.argv[2], "value", d["value"], "fwd97 %.1f inv97 %.1f (inv01 %.1f) | fwd53 %.1f (mct3 %.1f) inv53 %.1f (inv01 %.1f)" % (
    r["span_us"], r["inverse"]["span_us"], r["inverse"]["launches"][-1]["us"], r53["forward"]["span_us"],
    r53["forward"]["launches"][0]["us"], r53["inverse"]["span_us"], r53["inverse"]["launches"][-1]["us"]))
PY
done
done
unset GRKGPU_INV01_WPE GRKGPU_MCT3_WPE
export GRKGPU_INV01_WPE=6 GRKGPU_MCT3_WPE=5
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dwt or decode or 53 or encode" > gpurun_out/$T/pytest.txt 2>&1; tail -1 gpurun_out/$T/pytest.txt
