# 64-bit shift issue rate (scripts/shiftrate.hip), then the decoder bit-window A/B (GRKGPU_T1_NARROW 0 | 1)
set -o pipefail
T=${1:-r05n2}
mkdir -p gpurun_out/$T
timeout -k 10 60 ./scripts/shiftrate | tee gpurun_out/$T/shiftrate.txt || exit 1
bash scripts/gpu_env_ab.sh $T GRKGPU_T1_NARROW 0 1
