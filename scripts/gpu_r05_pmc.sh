#!/bin/bash
# SQ + HBM counter passes over the forward-DWT kernels of 3 8K encodes, one
# rocprofv3 run per counter group and setting.
#   bash scripts/gpu_r05_pmc.sh TAG "97 pair_kernel=0" "97 -" ...   (ENV=... prefix allowed: "GRKGPU_PAIR_CHUNK=8 97 -")
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for SPEC in "$@"; do
  i=$((i+1))
  for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
    n=$(echo $G | cut -c1-5)
    ENVS=$(echo "$SPEC" | tr ' ' '\n' | grep '=' | grep -v '^[a-z]' | tr '\n' ' ')
    ARGS=$(echo "$SPEC" | tr ' ' '\n' | grep -v '^[A-Z_]*=' | grep -v '^-$' | tr '\n' ' ')
    mkdir -p $OUT/s$i
    ( export $ENVS; timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $OUT/s$i/$n -o run -- python3 -u scripts/dwt_enc_once.py $ARGS > $OUT/s$i/$n.log 2>&1 ) || { echo "pmc $SPEC $G failed"; tail -5 $OUT/s$i/$n.log; exit 1; }
  done
  echo "s$i: $SPEC"
done
