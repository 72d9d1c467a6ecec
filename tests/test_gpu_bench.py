"""The bench.py contract on the GPU: one short run (2 frames in flight, one
timed step) must print exactly one JSON line with the driver's keys, the
roofline and cpu_baseline objects, and the PCIe-inclusive leg beside the
HBM-resident value.  A subprocess, one at a time (the bench re-launches
itself with more hardware queues before touching the GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_keeps_the_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1",
                        "--concurrency", "2", "--no-cpu-baseline"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "pcie_inclusive"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 1 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert "workload" in d["config"] and "model" not in d["config"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # frac = B_DWT over the device time of the frame's level sequence (span_us);
    # the per-launch breakdown sums to dwt_us
    assert abs(rf["algorithmic_bytes"] / (rf["span_us"] * 1e-6) / 1e9 - rf["achieved"]) < 0.5
    assert abs(sum(x["us"] for x in rf["launches"]) - rf["dwt_us"]) < 0.05
    inv = rf["inverse"]
    assert 0 < inv["frac"] < 1 and inv["launches"] and sum(x["algorithmic_bytes"] for x in inv["launches"]) == \
        rf["algorithmic_bytes"]
    assert d["cpu_baseline"] is None  # --no-cpu-baseline
    assert d["pcie_inclusive"]["value"] > 0 and d["pcie_inclusive"]["steps"] == 1


def test_bench_two_ranks_on_one_gpu():
    """--gpus 2 launches two ranks itself (torch.distributed.run); rank r takes
    device LOCAL_RANK % device_count, so on a one-GPU lease both share it;
    the timing barrier / max reduction go over gloo.  One JSON line (rank 0)
    with n_gpus 2 and the frames of both ranks in value."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "1", "--concurrency", "2", "--no-cpu-baseline", "--no-pcie"], cwd=ROOT, capture_output=True,
                       text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["frames_per_step_per_gpu"] == 2
    assert d["cpu_baseline"] is None and d["pcie_inclusive"] is None
    # value counts both ranks' frames over the slower rank's time
    px = 7680 * 4320
    assert abs(d["value"] - 2 * 2 * px * d["steps"] / (d["ms_per_step"] * 1e-3 * d["steps"]) / 1e6) < 0.01 * d["value"]
