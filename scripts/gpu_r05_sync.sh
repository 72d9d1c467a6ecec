# host waits through blocking-sync events (GRKGPU_BLOCKING_SYNC=1) vs hipStreamSynchronize: C5 and 8K lines, alternating
set -o pipefail
T=${1:-r05b}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
for v in 0 1; do
GRKGPU_BLOCKING_SYNC=$v timeout -k 10 400 python3 -u bench.py --workload c5 --steps 20 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/$T/c5_${v}_$r.json 2> gpurun_out/$T/c5_${v}_$r.err || { tail -30 gpurun_out/$T/c5_${v}_$r.err; exit 1; }
python3 - gpurun_out/$T/c5_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, dd = d["stage_ms"]["enccin"], d["stage_ms"]["deccin"]
print("c5 blocking", sys.argv[2], "value", d["value"], "enc t1 %.2f host_t2 %.2f rate %.2f packet %.2f passrec %.2f | dec t1 %.2f host_t2 %.2f" % (e["t1_ms"], e["host_t2_ms"], e["rate_ms"], e["packet_ms"], e["passrec_ms"], dd["t1_ms"], dd["host_t2_ms"]))
PY
GRKGPU_BLOCKING_SYNC=$v timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/$T/b8k_${v}_$r.json 2> gpurun_out/$T/b8k_${v}_$r.err || { tail -30 gpurun_out/$T/b8k_${v}_$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('8k blocking', sys.argv[2], 'value', d['value'], {k:(round(v['t1_ms'],1), round(v['host_t2_ms'],2)) for k,v in d['stage_ms'].items()})" gpurun_out/$T/b8k_${v}_$r.json $v
done
done
GRKGPU_BLOCKING_SYNC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1; tail -1 gpurun_out/$T/pytest.txt
