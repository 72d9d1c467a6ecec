#!/bin/bash
# PMC passes (one counter group per run) over the DWT stage probe.
set -o pipefail
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$C -o run -- python3 -u scripts/dwt_bench.py --stage > $OUT/$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
echo done
