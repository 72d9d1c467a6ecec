#!/bin/bash
# GPU box: HBM bytes (PMC FETCH_SIZE / WRITE_SIZE, one rocprofv3 --pmc pass
# each) of every kernel of scripts/enc_frames.py, for lib/ (A) and lib_ab/ (B).
#   bash scripts/gpu_pmc_ab.sh TAG "<enc_frames args>"
set -o pipefail
TAG=${1:-pmcab}
ARGS=${2:-3 97}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in A B; do
  if [ $v = B ]; then export GRKGPU_LIB=$PWD/grokimagecompression_amd/lib_ab/libgrk_mi355x.so; else unset GRKGPU_LIB; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/${v}_$C -o run -- python3 -u scripts/enc_frames.py $ARGS > $OUT/${v}_$C.log 2>&1 || { echo "pmc $v $C failed"; tail -5 $OUT/${v}_$C.log; exit 1; }
  done
  mkdir -p $OUT/$v && mv $OUT/${v}_FETCH_SIZE $OUT/$v/FETCH_SIZE && mv $OUT/${v}_WRITE_SIZE $OUT/$v/WRITE_SIZE
  python3 scripts/pmc_summary.py $OUT/$v $OUT/pmc_$v.json > /dev/null && echo "== $v" && python3 -c "
import json; d=json.load(open('$OUT/pmc_$v.json'))
rows=[(k,e) for k,v in d['kernels'].items() for e in v]
for k,e in sorted(rows, key=lambda r: -r[1]['bytes'])[:10]:
    print('%-44s grid %9d x%-3d read %9.1f MB write %9.1f MB per dispatch' % (k[:44], e['grid'], e['dispatches'], (e['read_bytes'] or 0)/1e6, (e['write_bytes'] or 0)/1e6))
"
done
