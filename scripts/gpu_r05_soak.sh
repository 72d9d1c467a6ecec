# soak: long bench runs on the final build (stability, sustained rate)
set -o pipefail
T=${1:-r05k2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/$T/b8k_60.json 2> gpurun_out/$T/b8k_60.err || { tail -20 gpurun_out/$T/b8k_60.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('8k 60 steps', d['value'], d['ms_per_step'], d['pcie_inclusive']['value'])" gpurun_out/$T/b8k_60.json
timeout -k 10 600 python3 -u bench.py --workload c5 --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/$T/c5_60.json 2> gpurun_out/$T/c5_60.err || { tail -20 gpurun_out/$T/c5_60.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['stage_ms']['enccin']; print('c5 60 steps', d['value'], d['ms_per_step'], 'enc t1', round(e['t1_ms'],2), 'host', round(e['host_t2_ms'],2))" gpurun_out/$T/c5_60.json
