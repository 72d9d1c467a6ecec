# the round's new GPU tests: marker fixtures (incl. conflicting tile-part COD / QCD),
# the held-views spare buffers, the grk_* API over the marker streams
set -o pipefail
T=${1:-r05n}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_grk_api.py -m gpu -x -q --timeout 300 --timeout-method thread -k "marker or view or mk_" > gpurun_out/$T/pytest.txt 2>&1; rc=$?; tail -15 gpurun_out/$T/pytest.txt; exit $rc
