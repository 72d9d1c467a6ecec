# wavefront-per-segment unstuff (GRKGPU_T1_UNSTUFF_WAVE=1): the GPU suite under it, then the bench A/B
set -o pipefail
T=${1:-r05u}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
GRKGPU_T1_UNSTUFF_WAVE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_full.txt 2>&1 || { tail -40 gpurun_out/$T/pytest_full.txt; exit 1; }
tail -1 gpurun_out/$T/pytest_full.txt
bash scripts/gpu_env_ab.sh ${T}ab GRKGPU_T1_UNSTUFF_WAVE 0 1 || exit 1
GRKGPU_T1_UNSTUFF_WAVE=1 GPU_MAX_HW_QUEUES=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-pcie --steps 2 --warmup 1 --concurrency 2 > gpurun_out/$T/prof_bench.json 2> gpurun_out/$T/prof.err || { tail -20 gpurun_out/$T/prof.err; exit 1; }
python3 scripts/prof_summary.py gpurun_out/$T/prof gpurun_out/$T/kernel_stats.csv > /dev/null && head -8 gpurun_out/$T/kernel_stats.csv
