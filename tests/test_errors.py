"""Error behaviour on malformed input (the reference's fuzz-regression cases,
j2k.cpp:3380-3480 read_siz, :3829-3884 read_cod, :4075 read_qcd,
:6978-7025 read_SPCod_SPCoc): a malformed or unsupported codestream makes
the call fail with a GrkGpuError (grkgpu status != 0) -- never a crash, a
hang or a GPU fault -- and the codec keeps working afterwards.

CPU tests exercise the host header parser (grkgpu_read_header needs no GPU);
the gpu tests push truncated / corrupted tile data through the whole decoder.
"""
import struct

import numpy as np
import pytest

from conftest import GOLD, load_manifest

MAN = load_manifest()
NAMES = sorted(MAN)


def _cs(name):
    return open("%s/%s.j2k" % (GOLD, name), "rb").read()


def _marker(cs, code):
    """Offset of the first main-header marker `code` (SOC .. first SOT)."""
    pos = 2
    while pos + 4 <= len(cs):
        m, L = struct.unpack(">HH", cs[pos:pos + 4])
        if m == code:
            return pos
        if m == 0xFF90:  # first SOT: end of the main header
            break
        pos += 2 + L
    raise KeyError(hex(code))


def _patch(cs, off, fmt, value):
    b = bytearray(cs)
    struct.pack_into(fmt, b, off, value)
    return bytes(b)


def _grk():
    import grokimagecompression_amd as grk
    return grk


def _rejects(cs):
    grk = _grk()
    with pytest.raises(grk.GrkGpuError):
        grk.read_header(cs)


@pytest.mark.parametrize("name", NAMES)
def test_goldens_parse(name):
    d = _grk().read_header(_cs(name))
    h, w, c, bits = MAN[name]["shape"]
    assert (d.numcomps, d.x1 - d.x0, d.y1 - d.y0) == (c, w, h)


def test_truncated_main_header_rejected():
    for name in ("rgb12_I", "g8_off_tiles", "g16_128"):
        cs = _cs(name)
        sot = _marker(cs, 0xFF90)
        for n in range(sot):
            _rejects(cs[:n])


def test_siz_field_checks():
    cs = _cs("rgb8_128x96")
    siz = _marker(cs, 0xFF51)
    x1, y1, x0, y0 = struct.unpack(">IIII", cs[siz + 6:siz + 22])
    _rejects(_patch(cs, siz + 14, ">I", x1))          # x0 == x1: zero image size
    _rejects(_patch(cs, siz + 18, ">I", y1 + 5))      # y0 > y1
    _rejects(_patch(cs, siz + 22, ">I", 0))           # tdx == 0
    _rejects(_patch(cs, siz + 34, ">I", x0 + 1))      # tile origin right of the image origin
    _rejects(_patch(cs, siz + 38, ">H", 4))           # Csiz does not match the marker length
    _rejects(_patch(cs, siz + 38, ">H", 0))           # no components
    _rejects(_patch(cs, siz + 40, ">B", 16))          # 17-bit precision: unsupported
    _rejects(_patch(cs, siz + 41, ">B", 0))           # XRsiz 0
    _rejects(_patch(cs, siz + 2, ">H", 20))           # marker too short


def test_cod_qcd_field_checks():
    cs = _cs("g8_256")
    cod = _marker(cs, 0xFF52)
    p = cod + 4
    _rejects(_patch(cs, p + 1, ">B", 5))              # unknown progression order
    _rejects(_patch(cs, p + 2, ">H", 0))              # zero layers
    _rejects(_patch(cs, p + 5, ">B", 33))             # 34 resolutions
    _rejects(_patch(cs, p + 6, ">B", 9))              # 2^11-wide code-blocks
    _rejects(_patch(cs, p + 8, ">B", 0x40))           # HT code-block style
    _rejects(_patch(cs, p + 9, ">B", 2))              # qmfbid 2
    _rejects(_patch(cs, p, ">B", 1))                  # Scod: user precincts, but no precinct sizes
    _rejects(_patch(cs, p, ">B", 8))                  # unknown Scod bit
    _rejects(_patch(cs, cod + 2, ">H", 4))            # COD too short
    qcd = _marker(cs, 0xFF5C)
    _rejects(_patch(cs, qcd + 4, ">B", 1))            # scalar-derived: one step size, not the marker's 16
    _rejects(_patch(cs, qcd + 2, ">H", 2))            # QCD too short


def test_random_main_header_corruption_never_crashes():
    grk = _grk()
    rng = np.random.default_rng(7)
    for name in ("rgb12_I", "g8_off_tiles", "g8_n1"):
        cs = _cs(name)
        sot = _marker(cs, 0xFF90)
        for _ in range(3000):
            b = bytearray(cs)
            for pos in rng.integers(0, sot, size=int(rng.integers(1, 4))):
                b[pos] = int(rng.integers(0, 256))
            try:
                d = grk.read_header(bytes(b))
            except grk.GrkGpuError:
                continue
            assert 1 <= d.numcomps <= 16 and d.x1 > d.x0 and d.y1 > d.y0


# ---------------------------------------------------------------- GPU decode

def _decode_or_error(codec, cs):
    grk = _grk()
    try:
        out = codec.decompress(cs)
    except grk.GrkGpuError:
        return None
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rgb12_I", "g8_256", "g8_off_tiles", "g16_128"])
def test_truncated_tile_data(codec, name):
    """Cut the codestream anywhere inside the tile-parts: the decoder either
    reports the corruption (a cut packet header) or decodes what is there
    (overlong segments truncated as the reference does); never faults."""
    cs = _cs(name)
    sot = _marker(cs, 0xFF90)
    ref = np.load("%s/%s.dec.npy" % (GOLD, name))
    rng = np.random.default_rng(11)
    cuts = sorted(set([sot + 1, sot + 12, sot + 14, len(cs) - 2, len(cs) - 1] +
                      [int(v) for v in rng.integers(sot, len(cs), size=24)]))
    for n in cuts:
        out = _decode_or_error(codec, cs[:n])
        if out is not None:
            assert out.shape == ref.shape
    # only the EOC missing: every packet is whole, so the image is exact
    assert np.array_equal(codec.decompress(cs[:-2]), ref)
    # a cut inside the last packet: segments are truncated (T2.cpp:686-698),
    # the decode completes
    if name != "g8_off_tiles":   # single tile: the last packet is a large body
        assert codec.decompress(cs[:-40]).shape == ref.shape
    assert np.array_equal(codec.decompress(cs), ref)   # still healthy


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rgb12_I", "g8_256", "g16_uniform_64"])
def test_corrupted_tile_data(codec, name):
    """Random byte damage in packet headers and code-block bytes (the MQ
    decoder runs on garbage): an error or an image of the right shape."""
    cs = _cs(name)
    sot = _marker(cs, 0xFF90) + 14
    ref = np.load("%s/%s.dec.npy" % (GOLD, name))
    rng = np.random.default_rng(5)
    for _ in range(40):
        b = bytearray(cs)
        for pos in rng.integers(sot, len(cs) - 2, size=int(rng.integers(1, 8))):
            b[pos] = int(rng.integers(0, 256))
        out = _decode_or_error(codec, bytes(b))
        if out is not None:
            assert out.shape == ref.shape
    assert np.array_equal(codec.decompress(cs), ref)


def test_encoder_parameter_checks():
    """grk_setup_encoder-style validation (j2k.cpp:1637-1660: resolutions in
    [1, 33], precision, code-block sizes; tile origin j2k.cpp:3466-3471), run
    through grkgpu_num_tiles, which shares the encoder's parameter setup."""
    grk = _grk()
    ok = grk.num_tiles((3, 64, 80), 8, grk.CParams.make())
    assert ok == 1
    assert grk.num_tiles((1, 100, 130), 8, grk.CParams.make(tiles=(32, 32))) == 4 * 5
    bad = [
        ((3, 64, 80), 8, grk.CParams.make(numresolution=0), (0, 0)),
        ((3, 64, 80), 8, grk.CParams.make(numresolution=34), (0, 0)),
        ((3, 64, 80), 8, grk.CParams.make(cblk=(128, 32)), (0, 0)),
        ((3, 64, 80), 8, grk.CParams.make(cblk=(48, 32)), (0, 0)),
        ((3, 64, 80), 8, grk.CParams.make(cblk=(2, 64)), (0, 0)),
        ((3, 64, 80), 17, grk.CParams.make(), (0, 0)),
        ((3, 64, 80), 0, grk.CParams.make(), (0, 0)),
        ((1, 0, 8), 8, grk.CParams.make(), (0, 0)),
        ((1, 64, 64), 8, grk.CParams.make(tiles=(16, 16), tile_offset=(5, 0)), (3, 0)),   # tx0 > x0
        ((1, 64, 64), 8, grk.CParams.make(tiles=(16, 16), tile_offset=(0, 0)), (20, 0)),  # x0 >= tx0 + tdx
        ((1, 4096, 4096), 8, grk.CParams.make(tiles=(8, 8)), (0, 0)),                    # 262144 tiles > 65535
    ]
    for shape, prec, params, off in bad:
        with pytest.raises(grk.GrkGpuError):
            grk.num_tiles(shape, prec, params, offset=off)
    import ctypes
    d = grk.ImageDesc()
    d.x1, d.y1, d.numcomps = 8, 8, 17                 # more components than the ABI carries
    for k in range(16):
        d.prec[k] = 8
    n = ctypes.c_uint32()
    assert grk.lib().grkgpu_num_tiles(ctypes.byref(d), ctypes.byref(grk.CParams.make()), ctypes.byref(n)) != 0


def test_dwt_options_checks():
    """grkgpu_set_dwt_options validates every field and the context manager
    restores the previous plan options (host code only)."""
    import ctypes
    grk = _grk()
    cur = grk.DwtOptions()
    grk.lib().grkgpu_get_dwt_options(ctypes.byref(cur))
    assert (cur.fuse_level0, cur.f01_rows, cur.f01_min_samples) == (-1, 4, 1 << 23)
    assert (cur.inv01, cur.inv01_min_samples) == (2, 1 << 23)
    with grk.dwt_options(f01_rows=6, fuse_level0=0):
        grk.lib().grkgpu_get_dwt_options(ctypes.byref(cur))
        assert (cur.f01_rows, cur.fuse_level0, cur.f01_min_samples) == (6, 0, 1 << 23)
    grk.lib().grkgpu_get_dwt_options(ctypes.byref(cur))
    assert (cur.f01_rows, cur.fuse_level0) == (4, -1)
    for kw in (dict(f01_rows=3), dict(f01_rows=8), dict(fuse_level0=2), dict(inv01=1), dict(inv01=3), dict(inv01=-1)):
        with pytest.raises(grk.GrkGpuError):
            with grk.dwt_options(**kw):
                pass
    grk.lib().grkgpu_get_dwt_options(ctypes.byref(cur))
    assert (cur.f01_rows, cur.fuse_level0) == (4, -1)


def _cut_manifest():
    import json
    return json.load(open("%s/manifest_cut.json" % GOLD))


def test_tile_walk_matches_reference():
    """The decoder's host side (grkgpu_walk_tiles: the tile-part walk, the
    packet headers and the code-block table, no device) on streams cut at
    ~1,400 positions (oracle/make_golden_cut.py: tile-part header edges,
    right after SOD, inside tile data, the tail), against the reference's own
    decodes of the same prefixes: it fails exactly where the reference fails
    (a stream ending inside a tile-part header, between a tile's tile-parts,
    inside a packet header -- but not inside a segment length, which the
    reference only warns about), and otherwise decodes exactly the tiles the
    reference's image holds (the others are zero)."""
    grk = _grk()
    man = _cut_manifest()
    ncuts = 0
    for name, rec in man.items():
        cs = _cs(name)
        for n, want in rec["cuts"].items():
            ncuts += 1
            try:
                got = grk.walk_tiles(cs[:int(n)])
            except grk.GrkGpuError:
                got = None
            if want == "error":
                assert got is None, (name, n, got)
                continue
            assert got is not None, (name, n)
            if want["tiles"] is not None:
                assert got == want["tiles"], (name, n, got, want["tiles"])
    assert ncuts > 1000


@pytest.mark.gpu
def test_cut_stream_matches_reference(codec):
    """GPU decodes of the ~1,400 cut streams of oracle/make_golden_cut.py
    against the reference's decodes of the same prefixes (Grok 5.1.0 built
    from /root/reference): an error exactly where the reference fails,
    otherwise the same image (SHA-256 of the decoded planes) -- tiles the
    stream never reaches zero, a tile cut inside its data decoded from what is
    there (T2.cpp:686-698), a tile decoded from the tile-parts read when the
    stream stops between them."""
    grk = _grk()
    man = _cut_manifest()
    import hashlib
    for name, rec in man.items():
        cs = _cs(name)
        for n, want in rec["cuts"].items():
            try:
                out = codec.decompress(cs[:int(n)])
            except grk.GrkGpuError:
                out = None
            if want == "error":
                assert out is None, (name, n)
                continue
            assert out is not None, (name, n)
            if isinstance(out, list):  # subsampled: per-component planes, flattened
                out = np.concatenate([np.asarray(p).ravel() for p in out])
            sha = hashlib.sha256(np.ascontiguousarray(out, dtype=np.int32).tobytes()).hexdigest()
            assert sha == want["sha"], (name, n)
    assert np.array_equal(codec.decompress(_cs("g8_tiles64")), np.load("%s/g8_tiles64.dec.npy" % GOLD))


@pytest.mark.gpu
def test_roi_shift_past_decoder_depth(codec):
    """An RGN shift raised so far that a code-block's bit-planes + shift reach
    31: the reference refuses the block (t1.cpp:1055-1060, "unsupported
    bpno_plus_one >= 31"); the GPU decoder, whose scratch holds 32 planes,
    must refuse it too -- a clean error, not a write past the block's
    scratch -- and stay healthy."""
    grk = _grk()
    cs = _cs("g8_roi_U5")
    rgn = _marker(cs, 0xFF5E)
    assert cs[rgn + 6] == 5  # Crgn (1 byte), Srgn, SPrgn = the shift
    for shift in (40, 60, 200):
        with pytest.raises(grk.GrkGpuError):
            codec.decompress(_patch(cs, rgn + 6, ">B", shift))
    ref = np.load("%s/g8_roi_U5.dec.npy" % GOLD)
    assert np.array_equal(codec.decompress(cs), ref)
