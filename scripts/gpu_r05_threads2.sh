# host pool cap A/B (GRKGPU_HOST_THREADS): 8K batch and C4 at 16 vs 8, C5 at 12 / 6, alternating
set -o pipefail
T=${1:-r05ht2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
pr() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sm = d.get("stage_ms", {})
hs = " ".join("%s t1 %.2f host %.2f" % (k, v.get("t1_ms", 0), v.get("host_t2_ms", 0)) for k, v in sm.items() if isinstance(v, dict))
print(sys.argv[2], "value %.1f" % d["value"], hs)
PY
}
for r in 1 2; do
for n in 16 8; do
GRKGPU_HOST_THREADS=$n timeout -k 10 400 python3 -u bench.py --steps 10 --no-cpu-baseline --no-pcie > gpurun_out/$T/b8k_${n}_$r.json 2> gpurun_out/$T/b8k_${n}_$r.err || { tail -30 gpurun_out/$T/b8k_${n}_$r.err; exit 1; }
pr gpurun_out/$T/b8k_${n}_$r.json "8k threads $n"
done
for n in 16 8; do
GRKGPU_HOST_THREADS=$n timeout -k 10 400 python3 -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c4_${n}_$r.json 2> gpurun_out/$T/c4_${n}_$r.err || { tail -30 gpurun_out/$T/c4_${n}_$r.err; exit 1; }
pr gpurun_out/$T/c4_${n}_$r.json "c4 threads $n"
done
for n in 12 6; do
GRKGPU_HOST_THREADS=$n timeout -k 10 400 python3 -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c5_${n}_$r.json 2> gpurun_out/$T/c5_${n}_$r.err || { tail -30 gpurun_out/$T/c5_${n}_$r.err; exit 1; }
pr gpurun_out/$T/c5_${n}_$r.json "c5 threads $n"
done
done
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
