#!/bin/bash
# GPU box: parity suite; DWT per-level times of the in-tree library vs lib_ab/;
# HBM-traffic PMC passes of the bench.  Usage: bash scripts/gpu_ab_dwt_pmc.sh TAG
set -o pipefail
TAG=${1:-abdwt}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for v in A B A B; do
  if [ $v = B ]; then L="GRKGPU_LIB=$PWD/grokimagecompression_amd/lib_ab/libgrk_mi355x.so"; else L="GRKGPU_NONE=1"; fi
  bash scripts/dwt_levels.sh $TAG/lev_$v$RANDOM $L > $OUT/lev.log 2>&1 || { echo "levels $v failed"; tail $OUT/lev.log; exit 1; }
  echo "== $v"; grep -E "fwd01|k_dwt_fwd<true" $OUT/lev.log
done
bash scripts/pmc_bench.sh $TAG/pmc > /dev/null || { echo "pmc failed"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/pmc/pmc_summary.json'))
for k,v in d['kernels'].items():
  if 't1' in k or 'fwd01' in k:
    for e in v: print('%-40s read %.1f MB write %.1f MB' % (k[:40], (e['read_bytes'] or 0)/1e6, (e['write_bytes'] or 0)/1e6))"
