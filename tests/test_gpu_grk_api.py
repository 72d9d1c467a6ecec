"""The grk_* C API drop-in (include/grk_api.h): the SAME
driver source that regenerates the golden fixtures with the reference's
libgrok (oracle/ref_driver.cpp: grk_compress's / grk_decompress's calls and
option mapping), compiled against the reference's grok.h and linked against
OUR grokimagecompression_amd/lib/libgrok.so instead (oracle/_ref/
ref_driver_mi355x, oracle/ref.mk).  Every golden case must come out
byte-identical on encode and sample-identical on decode -- including -r
(reduce) and -l (layers) decodes -- i.e. an application written against Grok's
API gets the reference's results from the MI355X path by relinking.

CPU part: the library exports the reference's whole grk_* function set.
"""
import hashlib
import json
import os
import struct
import subprocess

import numpy as np
import pytest

import synth
from conftest import GOLD, ROOT, load_manifest

MAN = load_manifest()
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver_mi355x")
LIB = os.path.join(ROOT, "grokimagecompression_amd", "lib", "libgrok.so")

# every GRK_API function of the reference's grok.h (v5.1.0)
REFERENCE_API = """grk_buffer_delete grk_buffer_new grk_create_compress grk_create_decompress grk_decode
grk_decode_tile_data grk_deinitialize grk_destroy_codec grk_destroy_cstr_index grk_destroy_cstr_info grk_dump_codec
grk_encode grk_encode_with_plugin grk_end_compress grk_end_decompress grk_get_cstr_index grk_get_cstr_info
grk_get_decoded_tile grk_image_all_components_data_free grk_image_create grk_image_destroy
grk_image_single_component_data_alloc grk_image_single_component_data_free grk_initialize grk_plugin_batch_decode
grk_plugin_batch_encode grk_plugin_cleanup grk_plugin_decode grk_plugin_encode grk_plugin_get_debug_state
grk_plugin_init grk_plugin_init_batch_decode grk_plugin_is_batch_complete grk_plugin_load grk_plugin_stop_batch_decode
grk_plugin_stop_batch_encode grk_read_header grk_read_tile_header grk_set_decode_area
grk_set_default_decoder_parameters grk_set_default_encoder_parameters grk_set_error_handler grk_set_info_handler
grk_set_warning_handler grk_setup_decoder grk_setup_encoder grk_start_compress grk_stream_create
grk_stream_create_file_stream grk_stream_create_mapped_file_read_stream grk_stream_create_mem_stream
grk_stream_destroy grk_stream_get_write_mem_stream_length grk_stream_set_read_function grk_stream_set_seek_function
grk_stream_set_user_data grk_stream_set_user_data_length grk_stream_set_write_function
grk_stream_set_zero_copy_read_function grk_version grk_write_tile grk_set_MCT""".split()


def test_library_exports_reference_api():
    if not os.path.exists(LIB):
        pytest.skip("libgrok.so not built")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [f for f in REFERENCE_API if f not in syms]
    assert not missing, missing


def _need_driver():
    if not os.path.exists(DRIVER):
        pytest.skip("oracle/_ref/ref_driver_mi355x not built (needs /root/reference at build time)")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MAN))
def test_grk_api_encode_matches_reference(name, tmp_path):
    _need_driver()
    m = MAN[name]
    h, w, c, bits = m["shape"]
    img = synth.synth_image(h, w, c, bits, m["seed"], m["kind"])
    src, out = tmp_path / "in.i32", tmp_path / "out.j2k"
    np.ascontiguousarray(img, dtype="<i4").tofile(src)
    r = subprocess.run([DRIVER, "enc", str(src), str(out), str(w), str(h), str(c), str(bits), "0"] + m["args"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == open(f"{GOLD}/{name}.j2k", "rb").read()


def _dec(name, tmp_path, extra=()):
    out = tmp_path / "out.i32"
    r = subprocess.run([DRIVER, "dec", f"{GOLD}/{name}.j2k", str(out)] + list(extra), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    x0, y0, x1, y1, nc, prec, sgnd, cw, ch = map(int, r.stdout.splitlines()[0].split())
    return np.fromfile(out, dtype="<i4").reshape(nc, ch, cw), (x0, y0, x1, y1, prec, sgnd)


INDEX = json.load(open(f"{GOLD}/cstr_index.json"))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(INDEX))
def test_grk_cstr_index_matches_reference(name):
    """grk_get_cstr_index through our libgrok.so: after grk_read_header and
    after grk_decode, every field (main-header markers, the first SOT,
    per-tile SOT / header markers / SOD, tile-part start / header end / end)
    printed by the same driver equals the reference's output
    (oracle/make_golden_index.py) for every golden codestream."""
    _need_driver()
    r = subprocess.run([DRIVER, "index", f"{GOLD}/{name}"], capture_output=True, text=True, timeout=120)
    got = r.stdout if r.returncode == 0 else "error"
    assert got == INDEX[name]


SUB = json.load(open(f"{GOLD}/manifest_sub.json"))


@pytest.mark.gpu
@pytest.mark.parametrize("tag", sorted(SUB))
def test_grk_api_subsampled_matches_reference(tag, tmp_path):
    """Subsampled grk_images through grk_compress's library calls (driver -sub:
    per-component grk_image_cmptparm dx / dy) and grk_decode: the same bytes
    and the same per-component planes as the reference."""
    _need_driver()
    m = SUB[tag]
    cd = lambda v, s: -(-v // s)  # noqa: E731
    a = m["args"]
    off = tuple(int(v) for v in a[a.index("-d") + 1].split(",")) if "-d" in a else (0, 0)
    w, h = m["size"]
    planes = [synth.synth_image(cd(off[1] + h, dy) - cd(off[1], dy), cd(off[0] + w, dx) - cd(off[0], dx), 1,
                                m["bits"], m["seed"] + k, m["kind"])[0] for k, (dx, dy) in enumerate(m["subsampling"])]
    src, out = tmp_path / "in.i32", tmp_path / "out.j2k"
    with open(src, "wb") as f:
        for p in planes:
            f.write(np.ascontiguousarray(p, dtype="<i4").tobytes())
    sub = "/".join("%d,%d" % tuple(s) for s in m["subsampling"])
    r = subprocess.run([DRIVER, "enc", str(src), str(out), str(w), str(h), str(len(planes)), str(m["bits"]), "0"] +
                       a + ["-sub", sub], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == open(f"{GOLD}/{tag}.j2k", "rb").read()
    dec = tmp_path / "out.i32"
    r = subprocess.run([DRIVER, "dec", f"{GOLD}/{tag}.j2k", str(dec)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    z = np.load(f"{GOLD}/{tag}.dec.npz")
    ref = np.concatenate([z["c%d" % k].ravel() for k in range(len(planes))])
    assert np.array_equal(np.fromfile(dec, dtype="<i4"), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MAN))
def test_grk_api_decode_matches_reference(name, tmp_path):
    _need_driver()
    d, hdr = _dec(name, tmp_path)
    ref = np.load(f"{GOLD}/{name}.dec.npy")
    assert d.shape == ref.shape and np.array_equal(d, ref)
    m = MAN[name]
    h, w, c, bits = m["shape"]
    ox, oy = map(int, m["args"][m["args"].index("-d") + 1].split(",")) if "-d" in m["args"] else (0, 0)
    assert hdr == (ox, oy, ox + w, oy + h, bits, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("name,tag", sorted((n, t) for n in MAN for t in MAN[n].get("variants", {})))
def test_grk_api_decode_options_match_reference(name, tag, tmp_path):
    """cp_reduce / cp_layer through grk_setup_decoder: the reference's own
    decode with those options, samples and image header."""
    _need_driver()
    v = MAN[name]["variants"][tag]
    d, hdr = _dec(name, tmp_path, v["args"])
    ref = np.load(f"{GOLD}/{name}.{tag}.dec.npy")
    assert d.shape == ref.shape and np.array_equal(d, ref)
    assert list(hdr) == v["header"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,r", [("g8_off35", 1), ("g8_off35", 2), ("g8_off_tiles", 1)])
def test_grk_api_reduced_odd_origin(codec, name, r, tmp_path):
    """-r of an image whose origin is not a multiple of 2^r: the components
    sized ceil(size / 2^r), as grk_image_comp_header_update sizes them
    (image.cpp:124-155), the image header unreduced, the decoded samples
    from ceil(origin / 2^r) on and the extra row / column zero (the
    reference's is uninitialised, so no fixture holds it).  The samples equal
    the Python path's, itself checked against the oracle
    (test_gpu_parity.py::test_reduced_decode_matches_oracle)."""
    _need_driver()
    d, hdr = _dec(name, tmp_path, ["-r", str(r)])
    h, w, c, bits = MAN[name]["shape"]
    cd = lambda v: -(-v >> r)  # noqa: E731
    assert d.shape == (c, cd(h), cd(w))
    ox, oy = map(int, MAN[name]["args"][MAN[name]["args"].index("-d") + 1].split(","))
    assert hdr[:4] == (ox, oy, ox + w, oy + h)
    assert np.array_equal(d, codec.decompress(open(f"{GOLD}/{name}.j2k", "rb").read(), reduce=r))
    dh, dw = cd(oy + h) - cd(oy), cd(ox + w) - cd(ox)
    assert not d[:, dh:].any() and not d[:, :, dw:].any()


@pytest.mark.gpu
def test_grk_api_decode_area(tmp_path):
    """grk_set_decode_area: the window of the reference's full decode."""
    _need_driver()
    d, hdr = _dec("rgb12_I", tmp_path, ["-d", "10,7,60,50"])
    ref = np.load(f"{GOLD}/rgb12_I.dec.npy")
    assert np.array_equal(d, ref[:, 7:50, 10:60])
    assert hdr[:4] == (10, 7, 60, 50)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rgb12_I", "g8_256", "rgb8_r10_tiles"])
def test_grk_api_concurrent_codecs(name, tmp_path):
    """Four caller threads, each with its own grk_* codecs, encode and decode
    at the same time (the reference allows one codec per caller thread): every
    result equals the single-threaded one.  The library leases a GPU context
    per call (grok_api.cpp), so no two calls share arenas or result buffers."""
    _need_driver()
    if name not in MAN:
        pytest.skip("fixture %s absent" % name)
    m = MAN[name]
    h, w, c, bits = m["shape"]
    img = synth.synth_image(h, w, c, bits, m["seed"], m["kind"])
    src = tmp_path / "in.i32"
    np.ascontiguousarray(img, dtype="<i4").tofile(src)
    r = subprocess.run([DRIVER, "mt", str(src), f"{GOLD}/{name}.j2k", str(w), str(h), str(c), str(bits), "0", "4",
                        "6"] + m["args"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr


# ---- tile streaming: grk_write_tile / grk_read_tile_header / grk_decode_tile_data /
# grk_get_decoded_tile, through the reference's own tile programs restated in
# oracle/tile_driver.cpp and linked against our libgrok.so.  Fixtures:
# oracle/make_tile_golden.py (the same driver linked against the reference).
TILE_DRIVER = os.path.join(ROOT, "oracle", "_ref", "tile_driver_mi355x")
with open(os.path.join(GOLD, "tiles.json")) as _f:
    TILES = json.load(_f)


def _sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _tile_run(*args):
    if not os.path.exists(TILE_DRIVER):
        pytest.skip("oracle/_ref/tile_driver_mi355x not built (needs /root/reference at build time)")
    r = subprocess.run([TILE_DRIVER] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr


def _tiles(path):
    out, a = {}, open(path, "rb").read()
    o = 0
    while o < len(a):
        h = struct.unpack_from("<7Q", a, o)
        out[h[0]] = (list(h), a[o + 56:o + 56 + h[6]])
        o += 56 + h[6]
    return out


@pytest.mark.parametrize("name", sorted(TILES))
def test_tile_fixture_integrity(name):
    assert _sha(os.path.join(GOLD, "tiles", name + ".j2k")) == TILES[name]["j2k_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(TILES))
def test_write_tile_matches_reference(name, tmp_path):
    """test_tile_encoder (tte*): grk_start_compress, grk_write_tile per tile,
    grk_end_compress -- the codestream is the reference's, byte for byte."""
    out = tmp_path / "t.j2k"
    args = TILES[name]["args"]
    _tile_run("enc", *[out if a == "OUT" else a for a in args], *([] if "OUT" in args else [out]))
    assert _sha(out) == TILES[name]["j2k_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(TILES))
def test_tile_decode_matches_reference(name, tmp_path):
    """test_tile_decoder (ttd*): grk_read_tile_header / grk_decode_tile_data
    over the reference's codestream, without a decode area: identical tile
    sequence, headers and samples.  With the ttd area: identical tile sequence
    and headers, and each tile's samples equal to its full decode (the
    reference's own samples there are not the tile's -- see tiles.json)."""
    m = TILES[name]
    j2k = os.path.join(GOLD, "tiles", name + ".j2k")
    full, area = tmp_path / "full.bin", tmp_path / "area.bin"
    _tile_run("dec", 0, 0, 0, 0, j2k, full)
    assert os.path.getsize(full) == m["full_bytes"] and _sha(full) == m["full_sha256"]
    _tile_run("dec", *m["area"], j2k, area)
    got, ref = _tiles(area), _tiles(full)
    assert [h for h, _ in got.values()] == m["area_tiles"]
    for t, (_, data) in got.items():
        assert data == ref[t][1], t


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(TILES))
def test_random_tile_access_matches_reference(name, tmp_path):
    """j2k_random_tile_access (rta*): grk_get_decoded_tile for the first, last
    and two middle tiles, each on a fresh decompressor."""
    out = tmp_path / "rta.bin"
    _tile_run("rta", os.path.join(GOLD, "tiles", name + ".j2k"), out)
    assert os.path.getsize(out) == TILES[name]["rta_bytes"] and _sha(out) == TILES[name]["rta_sha256"]
