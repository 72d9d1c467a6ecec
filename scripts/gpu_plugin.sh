#!/bin/bash
# GPU box: plugin-path parity + GPU parity of the newest fixtures + reference driver check
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 oracle/_ref/ref_driver bench tests/golden/../../gpurun_out/none 2>/dev/null; true
python - > gpurun_out/refdrv_diag.txt 2>&1 <<'PY'
import subprocess, numpy as np, sys
sys.path.insert(0, "tests/golden")
import synth
img = synth.synth_image(256, 256, 3, 8, 1, "smooth")
np.ascontiguousarray(img, dtype="<i4").tofile("/tmp/rd.i32")
r = subprocess.run(["oracle/_ref/ref_driver", "bench", "/tmp/rd.i32", "256", "256", "3", "8", "0", "16", "1"],
                   capture_output=True, text=True, timeout=120)
print("rc", r.returncode); print("out", r.stdout); print("err", r.stderr[-3000:])
PY
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_plugin.py \
  tests/test_plugin_abi.py "tests/test_gpu_parity.py" -k "plugin or init or prec_r or poc_r or exports or registration" \
  > gpurun_out/pytest_plugin.txt 2>&1
rc=$?
tail -5 gpurun_out/pytest_plugin.txt
exit $rc
