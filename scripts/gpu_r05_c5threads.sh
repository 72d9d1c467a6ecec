# C5 lines with the host pool capped at 16 / 8 / 4 threads (GRKGPU_HOST_THREADS), alternating
set -o pipefail
T=${1:-r05ht}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
for n in 16 8 4; do
GRKGPU_HOST_THREADS=$n timeout -k 10 400 python3 -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c5_${n}_$r.json 2> gpurun_out/$T/c5_${n}_$r.err || { tail -30 gpurun_out/$T/c5_${n}_$r.err; exit 1; }
python3 - gpurun_out/$T/c5_${n}_$r.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, dd = d["stage_ms"]["enccin"], d["stage_ms"]["deccin"]
print("threads", sys.argv[2], "value %.1f" % d["value"], "enc t1 %.2f host_t2 %.2f rate %.2f pkt %.2f passrec %.2f | dec t1 %.2f host_t2 %.2f" % (e["t1_ms"], e["host_t2_ms"], e["rate_ms"], e["packet_ms"], e["passrec_ms"], dd["t1_ms"], dd["host_t2_ms"]))
PY
done
done
