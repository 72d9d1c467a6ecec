# C5 host pool A/B (GRKGPU_POOL_BUSY_SERIAL 0 | 1, three alternating rounds),
# then the T1 SQ counters with the batch's block packing
set -o pipefail
T=${1:-r05c}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2 3; do
for v in 0 1; do
GRKGPU_POOL_BUSY_SERIAL=$v timeout -k 10 400 python3 -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c5_${v}_$r.json 2> gpurun_out/$T/c5_${v}_$r.err || { tail -30 gpurun_out/$T/c5_${v}_$r.err; exit 1; }
python3 - gpurun_out/$T/c5_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, dd = d["stage_ms"]["enccin"], d["stage_ms"]["deccin"]
print("busy_serial", sys.argv[2], "value", d["value"], "enc t1 %.2f host_t2 %.2f rate %.2f form %.2f | dec t1 %.2f host_t2 %.2f" % (
    e["t1_ms"], e["host_t2_ms"], e["rate_ms"], e["rate_form_ms"], dd["t1_ms"], dd["host_t2_ms"]))
PY
done
done
bash scripts/gpu_sq.sh ${T}_sq || exit 1
