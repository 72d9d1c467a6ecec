# model conditional reads v2 + register MRP contexts: GPU suite, HBM counters,
# then the decoder A/B (GRKGPU_T1_MRP_REG 0 | 1, alternating)
set -o pipefail
T=${1:-r05h}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_full.txt 2>&1 || { tail -40 gpurun_out/$T/pytest_full.txt; exit 1; }
tail -1 gpurun_out/$T/pytest_full.txt
bash scripts/pmc_bench.sh ${T}_pmc > /dev/null || exit 1
python3 - gpurun_out/${T}_pmc/pmc_summary.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
for k, v in b["kernels"].items():
    if "t1" in k or "mq" in k:
        print(k, [(e["dispatches"], round(e["read_bytes"] / 1e6), round(e["write_bytes"] / 1e6)) for e in v])
PY
bash scripts/gpu_env_ab.sh ${T}ab GRKGPU_T1_MRP_REG 0 1
