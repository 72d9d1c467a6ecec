set -o pipefail
T=${1:-r05d}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
GRKGPU_PAIR_CHUNK=80 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pair_stage" > gpurun_out/$T/pytest80.txt 2>&1 || { tail -30 gpurun_out/$T/pytest80.txt; exit 1; }
tail -2 gpurun_out/$T/pytest80.txt
for ch in 8 80; do
GRKGPU_PAIR_CHUNK=$ch timeout -k 10 300 python3 -u scripts/dwt_pair_probe.py - pair_waves=3 pair_waves=4 pair_rows=62 pair_rows=94 pair_waves=3,pair_rows=62 pair_waves=3,pair_rows=126 > gpurun_out/$T/probe$ch.txt 2>&1 || { tail -30 gpurun_out/$T/probe$ch.txt; exit 1; }
done
