#!/bin/bash
# The GPU-box runs behind the measurements in DESIGN.md / profiles/, one
# script with a mode per kind of run (each GPU step under its own timeout,
# the first failure ends the run).  Output: gpurun_out/TAG/.
#
#   bash scripts/gpu_run.sh final TAG      three C5 lines, the default 8K line, the 8K line on
#                                          uniform-noise frames (worst case), C4, the -m gpu suite, smoke
#   bash scripts/gpu_run.sh lines TAG [WL ...]   bench lines of the named workloads
#                                          (8k | 8k-uniform | 8k-const | c5 | c4 | g2; default 8k c5 c4)
#   bash scripts/gpu_run.sh prof TAG       rocprofv3 --kernel-trace --stats of a short bench run, the
#                                          roofline check against it, then the HBM counter passes (pmc_bench.sh)
#   bash scripts/gpu_run.sh sq TAG         SQ counters of the T1 kernels (gpu_sq.sh)
#   bash scripts/gpu_run.sh ab TAG         library A/B: lib/ vs lib_ab/ (probe_perf 8k + default line), ROUNDS rounds
#   bash scripts/gpu_run.sh env TAG VAR v1 v2 ...   an environment switch on the 8K line, two alternating rounds
#   bash scripts/gpu_run.sh soak TAG       60-step 8K and C5 lines
#   bash scripts/gpu_run.sh dwtpmc TAG "97 pair_kernel=0" "97 -" ...   SQ + HBM counter passes over the
#                                          forward-DWT kernels of 3 8K encodes (scripts/dwt_enc_once.py), one
#                                          rocprofv3 --pmc run per counter group and spec (ENV=V words allowed)
set -o pipefail
MODE=$1; TAG=${2:-$1}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp

# one-line summary of a bench JSON line
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = "%s value %.1f ms/step %.1f" % (sys.argv[2], d["value"], d["ms_per_step"])
r = d.get("roofline")
if r:
    s += " | dwt97 fwd frac %.3f (span %.1f us) inv %.3f" % (r["frac"], r.get("span_us", 0), r.get("inverse", {}).get("frac", 0))
if d.get("cpu_baseline"):
    s += " | cpu %.1f" % d["cpu_baseline"]["value"]
for k, v in sorted(d.get("stage_ms", {}).items()):
    if isinstance(v, dict) and "t1_ms" in v:
        s += " | %s t1 %.2f host_t2 %.2f" % (k, v["t1_ms"], v.get("host_t2_ms", 0))
print(s)
PY
}

# bench.py under a timeout; $1 = output name, the rest = bench.py arguments
bench() { local n=$1; shift
  timeout -k 10 500 python3 -u bench.py "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -30 $OUT/$n.err; exit 1; }
  summ $OUT/$n.json $n
}

line() {
  case $1 in
    8k) bench bench_8k ;;
    8k-uniform) bench bench_8k_uniform --data uniform ;;
    8k-const) bench bench_8k_const --data const ;;
    c5) bench bench_c5_$2 --workload c5 --steps 10 --warmup 2 ;;
    c4) bench bench_c4 --workload c4 --steps 5 --warmup 2 ;;
    g2) bench bench_g2 --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline ;;
    *) echo "unknown workload $1"; exit 2 ;;
  esac
}

case $MODE in
  final)
    for r in 1 2 3; do line c5 $r; done
    line 8k
    line 8k-uniform
    line c4
    timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
    tail -1 $OUT/pytest_gpu.txt
    timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
    tail -1 $OUT/smoke.txt
    ;;
  lines)
    WLS=${@:-8k c5 c4}
    i=0
    for w in $WLS; do i=$((i+1)); line $w $i; done
    ;;
  prof)
    GPU_MAX_HW_QUEUES=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-pcie --steps 2 --warmup 1 --concurrency 2 > $OUT/bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
    python3 scripts/prof_summary.py $OUT/prof $OUT/kernel_stats.csv > /dev/null
    python3 scripts/roofline_check.py $OUT/prof $OUT/bench.json | tee $OUT/roofline_check.txt
    bash scripts/pmc_bench.sh ${TAG}_pmc
    ;;
  sq)
    bash scripts/gpu_sq.sh $TAG
    ;;
  ab)
    AB=$PWD/grokimagecompression_amd/lib_ab/libgrk_mi355x.so
    for r in $(seq 1 ${ROUNDS:-2}); do
      for v in A B; do
        if [ $v = B ]; then export GRKGPU_LIB=$AB; else unset GRKGPU_LIB; fi
        timeout -k 10 200 python3 -u scripts/probe_perf.py 8k > $OUT/probe_${v}_$r.txt 2>&1 || { echo "probe $v failed"; tail $OUT/probe_${v}_$r.txt; exit 1; }
        bench bench_${v}_$r --no-cpu-baseline --no-pcie
      done
    done
    unset GRKGPU_LIB
    ;;
  env)
    V=$1; shift
    for r in 1 2; do
      for v in "$@"; do
        export $V=$v
        bench bench_${v}_$r --steps 10 --warmup 3 --no-cpu-baseline --no-pcie
      done
    done
    ;;
  soak)
    bench soak_8k_60 --steps 60 --warmup 3 --no-cpu-baseline
    bench soak_c5_60 --workload c5 --steps 60 --warmup 3 --no-cpu-baseline
    ;;
  dwtpmc)
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
    ;;
  *)
    echo "unknown mode $MODE"; exit 2 ;;
esac
