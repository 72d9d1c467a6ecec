# final build (host pool at half the CPU share; PCRD pass records prefetched): three C5 lines, the default 8K line, C4, the GPU suite, smoke
set -o pipefail
T=${1:-r05f5}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2 3; do
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 10 --warmup 2 > gpurun_out/$T/c5_$r.json 2> gpurun_out/$T/c5_$r.err || { tail -30 gpurun_out/$T/c5_$r.err; exit 1; }
python3 - gpurun_out/$T/c5_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, dd = d["stage_ms"]["enccin"], d["stage_ms"]["deccin"]
print(sys.argv[1], "value", d["value"], "cpu", d["cpu_baseline"]["value"], "enc t1 %.2f host_t2 %.2f rate %.2f | dec t1 %.2f host_t2 %.2f" % (e["t1_ms"], e["host_t2_ms"], e["rate_ms"], dd["t1_ms"], dd["host_t2_ms"]))
PY
done
timeout -k 10 400 python3 -u bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { tail -20 gpurun_out/$T/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench default', d['steps'], d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['inverse']['frac'], d['pcie_inclusive']['value'], d['cpu_baseline']['value'])" gpurun_out/$T/bench_default.json
timeout -k 10 400 python3 -u bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/$T/c4.json 2> gpurun_out/$T/c4.err || { tail -30 gpurun_out/$T/c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4', d['value'])" gpurun_out/$T/c4.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/$T/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/$T/pytest_gpu.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.txt 2>&1 || { tail -20 gpurun_out/$T/smoke.txt; exit 1; }
tail -1 gpurun_out/$T/smoke.txt
