"""The accelerator-plugin boundary: the REFERENCE host
(Grok 5.1.0's libgrok, oracle/_ref, built from source) loads OUR
libgrok_plugin.so through its own minpf loader and drives it exactly as
grk_compress's plugin_main does (grok.cpp:834-935, grk_compress.cpp:
2163-2305): grk_initialize(plugin_dir) -> grk_plugin_init ->
grk_plugin_encode -> (callback) grk_setup_encoder -> grk_start_compress ->
grk_encode_with_plugin(tile) -> grk_end_compress.  The plugin runs DC shift,
MCT, DWT, T1 and the per-pass distortion on the MI355X; the host runs rate
control and Tier-2 on the plugin's code-blocks (plugin_bridge.cpp:144-258).

Bar: the codestream the reference host writes from the plugin's blocks is
byte-identical to the one the reference writes alone (tests/golden/*.j2k),
for every rate-controlled fixture: 5/3 and 9/7, bisect and feasible
(-A 1), multi-layer with a lossless last layer, precincts / progressions /
SOP-EPH / tile-parts and both cinema profiles.  What the plugin does not take
must be declined (rc -1 -> the host encodes on its CPU path): tiles (the host
hands one plugin tile to every tile), a single layer without rate control
(the host forms that layer in make_single_lossless_layer BEFORE it copies the
plugin's passes in, TileProcessor.cpp:521 vs :537, so it would write an
empty layer), and fixed quality -q (its target uses tile->distotile, which
only the host's own T1 accumulates, T1Encoder.cpp:51).

The driver (oracle/_ref/ref_driver, built here by __graft_entry__.build())
travels to the GPU box with the tree; the test skips if it is absent.
"""
import os
import subprocess

import numpy as np
import pytest

import synth
from conftest import GOLD, ROOT, load_manifest

pytestmark = pytest.mark.gpu
MAN = load_manifest()
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
PLUGIN_DIR = os.path.join(ROOT, "grokimagecompression_amd", "lib")



def _handled(args):
    """Does the plugin take this grk_compress argument list?"""
    if "-t" in args:
        return False
    if "-M" in args and int(args[args.index("-M") + 1]) & 0x45:  # TERMALL / BYPASS / HT: multi-segment blocks
        return False
    if "-cinema2K" in args or "-cinema4K" in args:
        return True
    if "-q" in args:
        return False
    if "-r" in args:
        vals = [0.0 if float(v) == 1 else float(v) for v in args[args.index("-r") + 1].split(",")]
        return len(vals) > 1 or vals[0] > 0
    return False


HANDLED = sorted(n for n in MAN if _handled(MAN[n]["args"]))
DECLINED = sorted(n for n in MAN if not _handled(MAN[n]["args"]))


def _run(name, tmp_path):
    m = MAN[name]
    h, w, c, bits = m["shape"]
    img = synth.synth_image(h, w, c, bits, m["seed"], m["kind"])
    src = tmp_path / "in.i32"
    out = tmp_path / "out.j2k"
    np.ascontiguousarray(img, dtype="<i4").tofile(src)
    r = subprocess.run([DRIVER, "plugin", PLUGIN_DIR, str(src), str(out), str(w), str(h), str(c), str(bits)]
                       + list(m["args"]), capture_output=True, text=True, timeout=120)
    return r, out


@pytest.fixture(scope="module", autouse=True)
def _need_driver():
    if not os.path.exists(DRIVER):
        pytest.skip("oracle/_ref/ref_driver not built (needs /root/reference at build time)")
    if not os.path.exists(os.path.join(PLUGIN_DIR, "libgrok_plugin.so")):
        pytest.fail("libgrok_plugin.so missing: run __graft_entry__.build()")


@pytest.mark.parametrize("name", HANDLED)
def test_plugin_encode_matches_reference(name, tmp_path):
    r, out = _run(name, tmp_path)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == open(f"{GOLD}/{name}.j2k", "rb").read()


@pytest.mark.parametrize("name", [n for n in DECLINED if n in ("g8_tiles64", "rgb8_r10_tiles", "g8_64", "rgb12_I",
                                                                 "rgb8_poc", "g16_128")])
def test_plugin_declines(name, tmp_path):
    r, _ = _run(name, tmp_path)
    assert r.returncode == 3, r.stderr


# ---- decode: grk_decompress's plugin_main / decode_callback over plugin_decode ----

def _dec(name, tmp_path, extra=()):
    out = tmp_path / "out.i32"
    r = subprocess.run([DRIVER, "plugin-dec", PLUGIN_DIR, f"{GOLD}/{name}.j2k", str(out)] + list(extra),
                       capture_output=True, text=True, timeout=120)
    return r, out


def _planes(r, out):
    x0, y0, x1, y1, nc, prec, sgnd, w, h = map(int, r.stdout.split())
    return np.fromfile(out, dtype="<i4").reshape(nc, h, w)


DEC_CASES = ["g8_64", "g8_100x77", "g8_1x37", "g8_off35", "g8_off_tiles", "g16_128", "rgb8_128x96", "rgb8_nomct",
             "rgb12_96x80", "g8_64_I", "rgb12_I", "rgb12_tiles_I", "g16_I", "g8_r40_20_10", "rgb12_r30_10_1_I",
             "g12_r8_A1", "rgb8_prec_cprl", "rgb8_tp_C_cprl", "rgb8_poc", "g8_sop_eph", "rgb12_cinema4k",
             "rgb8_poc_r15_I"]


@pytest.mark.parametrize("name", DEC_CASES)
def test_plugin_decode_matches_reference(name, tmp_path):
    r, out = _dec(name, tmp_path)
    assert r.returncode == 0, r.stderr
    ref = np.load(f"{GOLD}/{name}.dec.npy")
    d = _planes(r, out)
    assert d.shape == ref.shape
    assert np.array_equal(d, ref)


@pytest.mark.parametrize("name,tag", sorted((n, t) for n in MAN for t in MAN[n].get("variants", {})))
def test_plugin_decode_options_match_reference(name, tag, tmp_path):
    """-r / -l through the host's decompress parameters (core.cp_reduce /
    core.cp_layer) against the reference's own decode with those options."""
    r, out = _dec(name, tmp_path, MAN[name]["variants"][tag]["args"])
    assert r.returncode == 0, r.stderr
    ref = np.load(f"{GOLD}/{name}.{tag}.dec.npy")
    d = _planes(r, out)
    assert d.shape == ref.shape
    assert np.array_equal(d, ref)


@pytest.mark.parametrize("name,win", [("rgb12_I", (10, 7, 60, 50)), ("g8_off_tiles", (20, 9, 170, 120)),
                                      ("rgb8_prec_r20_rpcl", (0, 0, 33, 150))])
def test_plugin_decode_window(name, win, tmp_path):
    """-d x0,y0,x1,y1 (parameters DA_*, grk_set_decode_area): the window of
    the reference's full decode."""
    r, out = _dec(name, tmp_path, ["-d", ",".join(map(str, win))])
    assert r.returncode == 0, r.stderr
    m = MAN[name]
    ox, oy = 0, 0
    if "-d" in m["args"]:
        ox, oy = map(int, m["args"][m["args"].index("-d") + 1].split(","))
    ref = np.load(f"{GOLD}/{name}.dec.npy")
    h, w = ref.shape[1:]
    x0, y0, x1, y1 = max(win[0], ox), max(win[1], oy), min(win[2], ox + w), min(win[3], oy + h)
    assert np.array_equal(_planes(r, out), ref[:, y0 - oy:y1 - oy, x0 - ox:x1 - ox])


def test_plugin_decode_declines_window_at_reduce(tmp_path):
    r, _ = _dec("rgb12_I", tmp_path, ["-r", "1", "-d", "0,0,20,20"])
    assert r.returncode == 3, r.stderr
