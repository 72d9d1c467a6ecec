set -o pipefail
O=gpurun_out/s10
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -u scripts/dwt_bench.py --sweep GRKGPU_DWT_FUSE=0 GRKGPU_DWT_FUSE=1 > $O/sweep.txt 2>&1
grep -v amdgpu.ids $O/sweep.txt
for s in 0 1; do
  GRKGPU_T1_SORT=$s timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_sort$s.json 2> $O/bench_sort$s.err || { tail -5 $O/bench_sort$s.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_sort$s.json')); print('sort=$s', d['value'], d['ms_per_step'], {k: round(v['t1_ms'],1) for k,v in d['stage_ms'].items()})"
done
