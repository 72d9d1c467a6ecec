set -o pipefail
mkdir -p gpurun_out/dw6
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "dwt or large_config" > gpurun_out/dw6/pytest.txt 2>&1 || { tail -30 gpurun_out/dw6/pytest.txt; exit 1; }
tail -1 gpurun_out/dw6/pytest.txt
timeout -k 10 600 python -u scripts/dwt_bench.py --sweep GRKGPU_DWT_STRIP=0 GRKGPU_DWT_STH=8,GRKGPU_DWT_NCH=4 GRKGPU_DWT_STH=8,GRKGPU_DWT_NCH=8 GRKGPU_DWT_STH=16,GRKGPU_DWT_NCH=2 GRKGPU_DWT_STH=16,GRKGPU_DWT_NCH=4 GRKGPU_DWT_STH=16,GRKGPU_DWT_NCH=4,GRKGPU_DWT_LAY=0 GRKGPU_DWT_STH=24,GRKGPU_DWT_NCH=2 GRKGPU_DWT_STRIP=0 > gpurun_out/dw6/sweep.txt 2>&1
grep -v amdgpu.ids gpurun_out/dw6/sweep.txt
