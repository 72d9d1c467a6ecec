# frames in flight (--concurrency) on the 8K batch with this round's decoder, two alternating rounds
set -o pipefail
T=${1:-r05q}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
for c in 12 16 20; do
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --concurrency $c --no-cpu-baseline --no-pcie > gpurun_out/$T/c${c}_$r.json 2> gpurun_out/$T/c${c}_$r.err || { tail -30 gpurun_out/$T/c${c}_$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('concurrency', sys.argv[2], 'round', sys.argv[3], 'value', d['value'])" gpurun_out/$T/c${c}_$r.json $c $r
done
done
