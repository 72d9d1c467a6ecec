set -o pipefail
mkdir -p gpurun_out/pv
cd scripts/probe && timeout -k 10 60 ./valu_rate > ../../gpurun_out/pv/valu.txt 2>&1; cd ../..
cat gpurun_out/pv/valu.txt
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pv/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/pv/avail.txt | sort -u | tr '\n' ' ' > gpurun_out/pv/sq_list.txt
cat gpurun_out/pv/sq_list.txt
