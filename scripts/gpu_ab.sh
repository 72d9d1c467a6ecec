# A/B bench: bash scripts/gpu_ab.sh TAG "ENV=.." "ENV=.." ...  (parity suite first)
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
[ -n "$NOTEST" ] || tail -1 $O/pytest.txt
i=0
for spec in "$@"; do
  i=$((i+1))
  (export $(echo $spec | tr ',' ' '); timeout -k 10 300 python -u bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --concurrency ${CONC:-12} > $O/b$i.json 2> $O/b$i.err) || { tail -5 $O/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$i.json')); print('$spec', d['value'], d['ms_per_step'], {k: round(v['t1_ms'],1) for k,v in d['stage_ms'].items()})"
done
