"""Pin the golden fixtures to the reference itself (CPU, build container only).

oracle/ref.mk compiles Grok v5.1.0's libgrok straight from /root/reference
(no CMake), oracle/ref_driver.cpp drives it through the grk_* C API, and
oracle/make_golden.py --check regenerates every committed fixture with it and
compares: codestream bytes, the reference decode, and the input image hash.
Together with tests/test_oracle_golden.py (restated oracle == fixtures) and
the -m gpu parity tests (HIP path == fixtures), this closes the chain
reference == fixtures == oracle == GPU.

Skipped where /root/reference does not exist (the GPU box).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HAVE_REF = os.path.isdir("/root/reference/src/lib/jp2")

pytestmark = pytest.mark.skipif(not HAVE_REF, reason="reference sources not present (GPU box)")


def _check(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "make_golden.py"), "--check", *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_reference_builds_and_exports_grk_api():
    subprocess.run(["make", "-s", "-f", "oracle/ref.mk", "-j8"], cwd=ROOT, check=True, timeout=900)
    lib = os.path.join(ROOT, "oracle", "_ref", "libgrok.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for s in ("grk_create_compress", "grk_setup_encoder", "grk_encode", "grk_decode", "grk_read_header",
              "grk_plugin_load", "grk_plugin_encode", "grk_plugin_decode"):
        assert s in syms


def test_small_fixtures_regenerate_bit_exact():
    out = _check()
    assert "mismatches 0" in out


def test_guard_bit_fixtures_regenerate():
    """tests/golden/*.gb<N>.*: goldens with patched QCD guard bits, decoded by
    the reference (oracle/make_golden_gbits.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "make_golden_gbits.py"), "--check"], cwd=ROOT,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_marker_fixtures_regenerate():
    """tests/golden/mk_*: COC / QCC / tile-part COD / QCD / RGN / PPM / PPT
    streams assembled from reference-encoded streams and decoded by the
    reference (oracle/make_golden_markers.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "make_golden_markers.py"), "--check"], cwd=ROOT,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_subsampled_fixtures_regenerate():
    """tests/golden/sub_*: subsampled-component images encoded and decoded by
    the reference (oracle/make_golden_sub.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "make_golden_sub.py"), "--check"], cwd=ROOT,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_index_fixtures_regenerate():
    """tests/golden/cstr_index.json: the reference's grk_get_cstr_index of
    every golden (oracle/make_golden_index.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "make_golden_index.py"), "--check"], cwd=ROOT,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_mct_fixtures_regenerate():
    """tests/golden/mct_*: custom-MCT streams encoded by the reference
    (oracle/make_golden_mct.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "make_golden_mct.py"), "--check"], cwd=ROOT,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_cstr_info_matches_reference():
    """grk_get_cstr_info of our libgrok.so (ref_driver_mi355x: the same driver
    relinked against it; header parsing needs no GPU) prints exactly what the
    reference's does for every golden and guard-bit fixture: tile grid,
    default coding style, per-component code-block / quantisation / precinct
    fields, with the reference's quirks (compno 0, byte-count precinct copy)."""
    import glob
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    ours = os.path.join(ROOT, "oracle", "_ref", "ref_driver_mi355x")
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.j2k")))
    assert len(files) > 50
    for f in files:
        a = subprocess.run([ref, "info", f], capture_output=True, text=True, timeout=60)
        b = subprocess.run([ours, "info", f], capture_output=True, text=True, timeout=60)
        if a.returncode != 0:  # a header the reference refuses (custom-MCT streams): ours refuses it too
            assert b.returncode != 0, f
            continue
        assert b.returncode == 0 and b.stdout == a.stdout, (f, a.stdout[:400], b.stdout[:400], b.stderr)


def test_c1_config_hash_regenerates():
    out = _check("--large", "--only", "C1_512_gray8")
    assert "C1_512_gray8 ok" in out


def test_plugin_abi_layout_matches_reference_headers():
    """include/grk_plugin_abi.h re-declares grok.h's plugin-boundary structs;
    oracle/abi/ compiles one offset/size table over the reference's headers
    and one over ours and compares them field by field."""
    subprocess.run(["make", "-s", "-f", "oracle/ref.mk", "-j8", "oracle/_ref/abi_check"], cwd=ROOT, check=True,
                   timeout=900)
    r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "abi_check")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert " 0 mismatches" in r.stdout


def test_oracle_nmsedec_tables_match_reference():
    """The oracle's distortion tables (restating the generator
    t1_generate_luts.cpp:290-318) equal the tables the reference ships and
    compiles (t1_part1/t1_luts.h lut_nmsedec_sig / sig0 / ref / ref0)."""
    import ctypes
    import re
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    got = np.zeros(512, np.int16)
    pyoracle.lib().orc_nmse_tables(got.ctypes.data_as(ctypes.c_void_p))
    txt = open("/root/reference/src/lib/jp2/t1/t1_part1/t1_luts.h").read()
    for k, name in enumerate(("lut_nmsedec_sig", "lut_nmsedec_sig0", "lut_nmsedec_ref", "lut_nmsedec_ref0")):
        body = re.search(name + r"\[[^\]]*\]\s*=\s*\{([^}]*)\}", txt).group(1)
        vals = [int(v, 0) for v in body.replace("\n", " ").split(",") if v.strip()]
        assert vals == [int(v) for v in got[128 * k:128 * (k + 1)]], name


def test_set_mct_size_mismatch_refused_at_setup(tmp_path):
    """grk_set_MCT's matrix is n x n for the n it was given; grk_setup_encoder
    of an image with another component count is refused (ours: an error
    before anything reaches the device, instead of reading past the
    allocation; grok_api.cpp map_cparams).  CPU only: setup never touches the
    GPU."""
    import numpy as np
    ours = os.path.join(ROOT, "oracle", "_ref", "ref_driver_mi355x")
    src, out = tmp_path / "in.i32", tmp_path / "out.j2k"
    np.zeros((3, 16, 16), dtype="<i4").tofile(src)
    r = subprocess.run([ours, "enc", str(src), str(out), "16", "16", "3", "8", "0", "-I",
                        "-mct", "1,0,0,1:0,0"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "custom MCT matrix (grk_set_MCT) of 2 components for an image of 3" in r.stderr
