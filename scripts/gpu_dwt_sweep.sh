set -o pipefail
O=gpurun_out/s14
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -u scripts/dwt_bench.py --sweep GRKGPU_MCT_NT=0 GRKGPU_MCT_NT=1 GRKGPU_DWT_BNT=1 GRKGPU_MCT_NT=1,GRKGPU_DWT_BNT=1 GRKGPU_MCT_NT=0 GRKGPU_MCT_NT=1 > $O/sweep.txt 2>&1
grep -v amdgpu.ids $O/sweep.txt
