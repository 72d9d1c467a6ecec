#!/bin/bash
# Run the bench (no CPU baseline, 3 steps) under several env settings; one line each.
# BENCH_ARGS inside a setting is passed to bench.py.
set -o pipefail
for E in "$@"; do
  echo "== $E"
  ( export $E; timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null ) | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print(d['value'], {k:(v['t1_ms'],v['dwt_ms']) for k,v in d['stage_ms'].items()})" || exit 1
done
