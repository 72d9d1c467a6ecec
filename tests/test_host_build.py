"""CPU-only checks: the HIP library builds for gfx950, loads, exports every
symbol include/grk_mi355x.h declares, fails loudly without a GPU; the T1
block coder compiled for the host matches the oracle bit-for-bit."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "grk_mi355x.h")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(grkgpu_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    import grokimagecompression_amd as grk
    if not os.path.exists(grk.LIB_PATH):
        grk.build()
    L = grk.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s


def test_library_is_gfx950_code_object():
    import grokimagecompression_amd as grk
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", grk.LIB_PATH], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(grk.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_cpu_fallback_without_gpu():
    import torch
    import grokimagecompression_amd as grk
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(grk.GrkGpuError):
        grk.Codec(0)


def test_t1_core_host_matches_oracle(oracle, tmp_path):
    exe = tmp_path / "test_t1_core"
    ob = os.path.join(ROOT, "oracle", "build")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-o", str(exe), os.path.join(ROOT, "tests/cpp/test_t1_core.cpp"),
                    "-L" + ob, "-lgrk_oracle", "-Wl,-rpath," + ob], check=True)
    r = subprocess.run([str(exe), "800"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]


def test_ict_term_identity():
    """grk_device.h ict_term: the forward ICT's int_fix_mul(r << 11, c)
    (mct.cpp:195-350, 64-bit product) equals floor((r c + 2) / 4) in 32-bit
    arithmetic for every DC-shifted sample of up to 16 bits."""
    import numpy as np
    r = np.arange(-(1 << 16), (1 << 16) + 1, dtype=np.int64)
    for c in (2449, 4809, 934, 1382, 2714, 4096, 3430, 666):
        ref = ((r << 11) * c + 4096) >> 13
        assert np.array_equal(ref, (r * c + 2) >> 2)
        assert np.abs(r * c).max() < 2 ** 31


# Layer-record digests of tests/cpp/pcrd_bench.cpp's synthetic cinema tile
# (algorithm, byte budget, seed, layers) as the full evaluation of every
# bisection probe gave them (t2.cpp before the incremental RateProbe; that
# code reproduced the reference's rate-controlled fixtures byte for byte).
PCRD_DIGESTS = [((0, "1.29e6", 1, 1), "b1bca82029ffdc6d"), ((0, "6e5", 2, 3), "169651092ad7142f"),
                ((1, "1.29e6", 1, 1), "78719fdaee4e6c99"), ((1, "6e5", 2, 3), "956b47338a3f1fed")]


def test_pcrd_incremental_probes_match_full_evaluation(tmp_path):
    exe = tmp_path / "pcrd_bench"
    c = os.path.join(ROOT, "grokimagecompression_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + c, "-o", str(exe), os.path.join(ROOT, "tests/cpp/pcrd_bench.cpp"),
                    os.path.join(c, "t2.cpp"), os.path.join(c, "codestream.cpp"), "-lpthread"], check=True)
    for (algo, budget, seed, layers), digest in PCRD_DIGESTS:
        # slopes 1: the per-block slope extremes precomputed as codec.cpp's pass-record fill does
        for slopes in ("0", "1"):
            r = subprocess.run([str(exe), str(algo), budget, str(seed), str(layers), "1", slopes], capture_output=True,
                               text=True, check=True)
            assert "digest %s" % digest in r.stdout, (algo, budget, seed, layers, slopes, r.stdout)


def test_pcrd_header_bound_holds(tmp_path):
    """The body_fits shortcut of the rate allocator (t2.cpp) skips a probe's
    packet simulation when the code-block bytes plus a bound on every packet
    header fit the budget; a checked build compares every simulated
    first-layer packet of a single-layer search with that bound:
    none may exceed it -- with one codeword segment per block, with TERMALL
    (a length per pass) and with BYPASS's segment pattern."""
    exe = tmp_path / "pcrd_bench_checked"
    c = os.path.join(ROOT, "grokimagecompression_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-DGRKGPU_CHECK_HEADER_UB", "-I" + c, "-o", str(exe),
                    os.path.join(ROOT, "tests/cpp/pcrd_bench.cpp"), os.path.join(c, "t2.cpp"),
                    os.path.join(c, "codestream.cpp"), "-lpthread"], check=True)
    for algo in ("0", "1"):
        for budget in ("1.29e6", "4e5", "3e6"):
            for terms in ("0", "1", "2"):
                r = subprocess.run([str(exe), algo, budget, "1", "1", "1", "1", terms], capture_output=True, text=True,
                                   check=True)
                m = re.search(r"header_ub checks (\d+) violations (\d+)", r.stdout)
                assert m, r.stdout
                assert int(m.group(1)) > 0 and int(m.group(2)) == 0, (algo, budget, terms, r.stdout)
