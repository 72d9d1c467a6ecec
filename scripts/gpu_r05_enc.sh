# Interleaved encoder scratch: the GPU suite, then the model occupancy A/B
# (GRKGPU_T1_MODEL_WPE 1 | 3, alternating), then the HBM counter passes.
set -o pipefail
T=${1:-r05e}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -40 gpurun_out/$T/pytest.txt; exit 1; }
tail -1 gpurun_out/$T/pytest.txt
bash scripts/gpu_env_ab.sh $T GRKGPU_T1_MODEL_WPE 1 3 || exit 1
bash scripts/pmc_bench.sh ${T}_pmc > /dev/null || exit 1
python3 - gpurun_out/${T}_pmc/pmc_summary.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
for k, v in b["kernels"].items():
    if "t1" in k or "mq" in k:
        print(k, [(e["dispatches"], round(e["read_bytes"] / 1e6), round(e["write_bytes"] / 1e6)) for e in v])
PY
