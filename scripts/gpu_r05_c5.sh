# C5 and 8K bench lines with stage_ms averaged over every timed frame
set -o pipefail
T=${1:-r05k}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2 3; do
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c5_$r.json 2> gpurun_out/$T/c5_$r.err || { tail -30 gpurun_out/$T/c5_$r.err; exit 1; }
python3 - gpurun_out/$T/c5_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, dd = d["stage_ms"]["enccin"], d["stage_ms"]["deccin"]
print(sys.argv[1], "value", d["value"], "frames", e["frames"], "enc t1 %.2f host_t2 %.2f rate %.2f form %.2f sim %.2f passrec %.2f packet %.2f | dec t1 %.2f host_t2 %.2f" % (
    e["t1_ms"], e["host_t2_ms"], e["rate_ms"], e["rate_form_ms"], e["rate_sim_ms"], e["passrec_ms"], e["packet_ms"], dd["t1_ms"], dd["host_t2_ms"]))
PY
done
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/$T/b8k.json 2> gpurun_out/$T/b8k.err || { tail -30 gpurun_out/$T/b8k.err; exit 1; }
python3 - gpurun_out/$T/b8k.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("8k value", d["value"], "frac", d["roofline"]["frac"], {k: (v["t1_ms"], v["host_t2_ms"], v["frames"]) for k, v in d["stage_ms"].items()})
PY
