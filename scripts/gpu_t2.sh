set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "${1:-encode_matches or decode_matches or large_config}" > gpurun_out/pytest_t2.txt 2>&1; rc=$?
tail -40 gpurun_out/pytest_t2.txt
exit $rc
