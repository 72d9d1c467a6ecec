set -o pipefail
T=${1:-r05f}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for ch in 1 2 3; do
GRKGPU_PAIR_CHUNK=$ch timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pair_stage" > gpurun_out/$T/pytest$ch.txt 2>&1 || { tail -30 gpurun_out/$T/pytest$ch.txt; exit 1; }
tail -1 gpurun_out/$T/pytest$ch.txt
done
for ch in 0 1 2 3; do
GRKGPU_PAIR_CHUNK=$ch timeout -k 10 300 python3 -u scripts/dwt_pair_probe.py - pair_rows=62 pair_rows=190 > gpurun_out/$T/probe$ch.txt 2>&1 || { tail -30 gpurun_out/$T/probe$ch.txt; exit 1; }
done
timeout -k 10 400 python -u -m pytest tests/test_errors.py tests/test_gpu_grk_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_api.txt 2>&1; tail -3 gpurun_out/$T/pytest_api.txt
