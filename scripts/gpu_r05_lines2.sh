# bench lines (C5 x2, C4, two ranks on one GPU), decoder SQ counters, plugin batch sweep
set -o pipefail
T=${1:-r05l}
bash scripts/gpu_r05_lines.sh $T || exit 1
timeout -k 10 600 python3 -u scripts/plugin_batch_sweep.py 24 4 8 16 > gpurun_out/$T/plugin_sweep.txt 2>&1; rc=$?; cat gpurun_out/$T/plugin_sweep.txt; exit $rc
