#!/bin/bash
# GPU box: lone-frame stage times (probe_perf 8k), per-level DWT kernel times
# (default and with the DC shift + MCT fused into level 0), and SQ counters of
# the T1 kernels on the lone 8K frame (two --pmc passes).
# Usage: bash scripts/gpu_t1_probe.sh TAG
set -o pipefail
TAG=${1:-t1probe}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list failed (ignored)"
timeout -k 10 200 python -u scripts/probe_perf.py 8k > $OUT/probe_8k.txt 2>&1 || { echo "probe failed"; tail $OUT/probe_8k.txt; exit 1; }
cat $OUT/probe_8k.txt
bash scripts/dwt_levels.sh $TAG/lev_default > /dev/null || { echo "levels failed"; exit 1; }
cat $OUT/lev_default/levels.txt
bash scripts/dwt_levels.sh $TAG/lev_fuse GRKGPU_DWT_FUSE=1 > /dev/null || { echo "levels fuse failed"; exit 1; }
cat $OUT/lev_fuse/levels.txt
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/sq$i -o run -- python3 -u scripts/probe_perf.py 8k > $OUT/sq$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/sq$i.log; exit 1; }
done
echo done
