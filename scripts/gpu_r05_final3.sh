# final build with the small-launch decoder: GPU suite, smoke, single-frame latency of every config, the bench line
set -o pipefail
T=${1:-r05x}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/$T/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/$T/pytest_gpu.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.txt 2>&1 || { tail -20 gpurun_out/$T/smoke.txt; exit 1; }
tail -1 gpurun_out/$T/smoke.txt
timeout -k 10 400 python3 -u scripts/probe_perf.py 512 4k 8k 16k > gpurun_out/$T/probe_all.txt 2>&1 || { tail -20 gpurun_out/$T/probe_all.txt; exit 1; }
grep -v "^  " gpurun_out/$T/probe_all.txt
timeout -k 10 400 python3 -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['frac'], d['roofline']['inverse']['frac'], d['cpu_baseline']['value'], d['t1']['lone_frame']['enc_t1_ms'], d['t1']['lone_frame']['dec_t1_ms'])" gpurun_out/$T/bench.json
