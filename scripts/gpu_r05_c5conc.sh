# C5 frames in flight (NS, default 12 / 16 / 20 / 24) with the half-share host pool, alternating (2 rounds)
set -o pipefail
T=${1:-r05cc}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
for n in ${NS:-12 16 20 24}; do
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --concurrency $n > gpurun_out/$T/c5_${n}_$r.json 2> gpurun_out/$T/c5_${n}_$r.err || { tail -30 gpurun_out/$T/c5_${n}_$r.err; exit 1; }
python3 - gpurun_out/$T/c5_${n}_$r.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, dd = d["stage_ms"]["enccin"], d["stage_ms"]["deccin"]
print("frames", sys.argv[2], "value %.1f" % d["value"], "enc t1 %.2f host_t2 %.2f rate %.2f | dec t1 %.2f host_t2 %.2f" % (e["t1_ms"], e["host_t2_ms"], e["rate_ms"], dd["t1_ms"], dd["host_t2_ms"]))
PY
done
done
