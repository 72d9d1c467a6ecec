"""GPU parity: the MI355X path (libgrk_mi355x.so via the C ABI) against the
reference's golden codestreams and the CPU oracle.

Bar: bit-exact for everything -- 5/3 and 9/7 codestream bytes (the encoder is
integer arithmetic end to end), 5/3 decode, and the 9/7 float decode (the
kernels reproduce the reference's operation order with no FMA contraction;
tolerance 0, i.e. max-abs 0 vs the reference decoder's output).
"""
import hashlib
import json

import numpy as np
import pytest

import synth
from conftest import GOLD, load_manifest, oracle_supported

pytestmark = pytest.mark.gpu
MAN = load_manifest()
LARGE = load_manifest(large=True)


def _img(m):
    h, w, c, bits = m["shape"]
    img = synth.synth_image(h, w, c, bits, m["seed"], m["kind"])
    assert synth.image_sha256(img) == m["image_sha256"]
    return img, bits


@pytest.mark.parametrize("name", sorted(MAN))
def test_encode_matches_reference_bytes(codec, name):
    import grokimagecompression_amd as grk
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    b = codec.compress(img, bits, p, offset=off)
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    assert len(b) == len(gold)
    assert b == gold


@pytest.mark.parametrize("name", ["rgb12_I", "g8_M4_termall", "rgb8_prec_r20_rpcl", "g16_M5_lazy_termall",
                                  "rgb12_cinema4k"])
@pytest.mark.parametrize("opts", [dict(t1_enc_sort=0), dict(t1_enc_sort=1, t1_enc_bpw=16)])
def test_encode_mq_lane_order_matches_reference(codec, name, opts):
    """The MQ coder's lanes take the blocks in the device work order
    (t1_enc_sort, default on) or in block order, packed 64 or 16 to a
    wavefront: the same codestream as the reference either way."""
    import grokimagecompression_amd as grk
    if name not in MAN:
        pytest.skip("fixture %s absent" % name)
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    with grk.dwt_options(**opts):
        b = codec.compress(img, bits, p, offset=off)
    assert b == open(f"{GOLD}/{name}.j2k", "rb").read()


def test_rate_control_stats(codec):
    """grkgpu_stats after a rate-controlled encode (the cinema golden): the
    PCRD bisection's probes, block evaluations (at least the first probe's
    full pass), probes decided without a packet simulation and precinct
    simulations are reported; a lossless single-layer encode runs no
    bisection."""
    import grokimagecompression_amd as grk
    m = MAN["rgb12_cinema4k"]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    codec.compress(img, bits, p, offset=off)
    st = codec.stats()
    assert st["rate_probes"] > 0 and st["rate_block_evals"] >= st["num_cblks"]
    assert st["rate_probes_skipped"] <= st["rate_probes"]
    # (the simple search's last probe ends it on the 0.001 tolerance before any simulation)
    assert st["rate_precinct_sims"] > 0 or st["rate_probes_skipped"] >= st["rate_probes"] - 1
    assert 0 <= st["rate_form_ms"] + st["rate_sim_ms"] <= st["rate_ms"] + 1e-3
    m = MAN["g8_64"]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    codec.compress(img, bits, p, offset=off)
    assert codec.stats()["rate_probes"] == 0


@pytest.mark.parametrize("name", sorted(MAN))
def test_decode_matches_reference(codec, name):
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    ref = np.load(f"{GOLD}/{name}.dec.npy")
    d = codec.decompress(gold)
    assert d.shape == ref.shape
    assert int(np.abs(d.astype(np.int64) - ref).max()) == 0


@pytest.mark.parametrize("name", ["rgb12_I", "g8_M4_termall", "g8_roi_U5", "rgb8_prec_r20_rpcl", "g12_M63",
                                  "rgb12_cinema4k", "g16_M5_lazy_termall"])
def test_decode_sorted_blocks_match_reference(codec, name):
    """t1_dec_sort: the decoder's lanes take the code-blocks in decreasing
    order of expected work (passes, bytes) -- blocks, codeword segments and
    ROI shifts permuted together; the image is the reference's."""
    import grokimagecompression_amd as grk
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    ref = np.load(f"{GOLD}/{name}.dec.npy")
    with grk.dwt_options(t1_dec_sort=1):
        d = codec.decompress(gold)
    assert np.array_equal(d, ref)
    with grk.dwt_options(t1_dec_sort=1, t1_dec_bpw=16):  # 16 blocks per wavefront
        d = codec.decompress(gold)
    assert np.array_equal(d, ref)


GBITS = sorted(json.load(open(f"{GOLD}/manifest_gbits.json")))


@pytest.mark.parametrize("tag", GBITS)
def test_decode_guard_bits_match_reference(codec, tag):
    """Goldens whose QCD guard-bit count is patched from Grok's 2 to 1 / 3
    (oracle/make_golden_gbits.py): band bit-planes = expn + guard bits - 1
    (j2k_read_SQcd_SQcc), so every code-block's bit-plane count moves; the
    decode equals the reference's own decode of the patched stream."""
    ref = np.load(f"{GOLD}/{tag}.dec.npy")
    d = codec.decompress(open(f"{GOLD}/{tag}.j2k", "rb").read())
    assert d.shape == ref.shape
    assert int(np.abs(d.astype(np.int64) - ref).max()) == 0


MARKERS = json.load(open(f"{GOLD}/manifest_markers.json"))


@pytest.mark.parametrize("tag", sorted(MARKERS))
def test_decode_marker_fixtures_match_reference(codec, tag):
    """Streams with main-header COC / QCC, tile-part COD / COC / QCD / QCC /
    RGN, PPM and PPT (oracle/make_golden_markers.py: spliced / rewritten from
    reference-encoded streams, decoded by the reference): per-tile and
    per-component numres, code-block and precinct sizes, progression, layer
    count, wavelet, quantisation and ROI shift, packet headers read from the
    packed-header segments -- bit-exact with the reference's decode."""
    m = MARKERS[tag]
    cs = open(f"{GOLD}/{tag}.j2k", "rb").read()
    assert hashlib.sha256(cs).hexdigest() == m["j2k_sha256"]
    if m.get("dec") == "error":
        with pytest.raises(Exception):
            codec.decompress(cs)
        return
    ref = np.load(f"{GOLD}/{tag}.dec.npy")
    d = codec.decompress(cs)
    assert d.shape == ref.shape
    assert int(np.abs(d.astype(np.int64) - ref).max()) == 0


MCT = json.load(open(f"{GOLD}/manifest_mct.json"))


@pytest.mark.parametrize("tag", sorted(MCT))
def test_custom_mct_encode_matches_reference(codec, tag):
    """Custom array-based MCT (grk_set_MCT; oracle/make_golden_mct.py): the
    13-bit fixed-point encoding matrix applied on the GPU after the DC shift
    (mct.cpp:429-475), the float inverse (matrix_inversion_f restated) in the
    CBD / MCT / MCC / MCO segments, Part-2 rsiz, rate control weighted by the
    inverse's column norms -- byte-identical to the reference.  Decoding is
    refused as the reference refuses it (COD MCT byte 2, j2k.cpp:3869)."""
    import grokimagecompression_amd as grk
    m = MCT[tag]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    b = codec.compress(img, bits, p, offset=off)
    gold = open(f"{GOLD}/{tag}.j2k", "rb").read()
    assert len(b) == len(gold)
    assert b == gold
    assert m["dec"] == "error"
    with pytest.raises(grk.GrkGpuError):
        codec.decompress(gold)


SUB = json.load(open(f"{GOLD}/manifest_sub.json"))


def _sub_planes(m):
    cd = lambda v, s: -(-v // s)  # noqa: E731
    a = m["args"]
    off = tuple(int(v) for v in a[a.index("-d") + 1].split(",")) if "-d" in a else (0, 0)
    w, h = m["size"]
    return [synth.synth_image(cd(off[1] + h, dy) - cd(off[1], dy), cd(off[0] + w, dx) - cd(off[0], dx), 1,
                              m["bits"], m["seed"] + k, m["kind"])[0] for k, (dx, dy) in enumerate(m["subsampling"])]


def _npz_planes(path, n):
    z = np.load(path)
    return [z["c%d" % k] for k in range(n)]


def assert_reduced_plane(x, ref, h, w):
    """A whole-image reduced decode: planes sized ceil(size / 2^r) as the
    reference sizes them (image.cpp:124-155), the decoded h x w samples from
    ceil(origin / 2^r) on.  With an origin that is not a multiple of 2^r the
    plane has one row / column more than that; the reference leaves it
    uninitialised (it differs from run to run), ours is zero."""
    assert x.shape == ref.shape
    assert h <= x.shape[0] <= h + 1 and w <= x.shape[1] <= w + 1
    assert np.array_equal(x[:h, :w], ref[:h, :w])
    assert not x[h:].any() and not x[:, w:].any()


@pytest.mark.parametrize("tag", sorted(SUB))
def test_subsampled_encode_decode_match_reference(codec, tag):
    """Subsampled components (SIZ XRsiz / YRsiz: 4:2:0, 4:2:2, 3x2, mixed
    1/2/4; oracle/make_golden_sub.py, encoded and decoded by the reference):
    each component coded on its own grid (TileComponent.cpp:193-196), the
    position-driven progressions stepping by dx / dy (PacketIter.cpp), MCT
    off when the first three differ (j2k.cpp:1963-1971).  The codestream is
    byte-identical to the reference's and the decode equals its decode."""
    import grokimagecompression_amd as grk
    m = SUB[tag]
    planes = _sub_planes(m)
    p, off = grk.CParams.from_cli(m["args"])
    b = codec.compress_subsampled(planes, m["bits"], tuple(m["size"]), [tuple(s) for s in m["subsampling"]], p,
                                  offset=off)
    gold = open(f"{GOLD}/{tag}.j2k", "rb").read()
    assert hashlib.sha256(gold).hexdigest() == m["j2k_sha256"]
    assert b == gold
    ref = _npz_planes(f"{GOLD}/{tag}.dec.npz", len(planes))
    d = codec.decompress(gold)
    assert len(d) == len(ref)
    for a, r in zip(d, ref):
        assert a.shape == r.shape and np.array_equal(a, r)
    if m["lossless"]:
        assert all(np.array_equal(a, s) for a, s in zip(d, planes))


SUB_VARIANTS = sorted((t, v) for t in SUB for v in SUB[t].get("variants", {}))


@pytest.mark.parametrize("tag,vt", SUB_VARIANTS)
def test_subsampled_decode_options_match_reference(codec, tag, vt):
    """-r / -l / -d decodes of subsampled streams: every component's plane on
    its grid, ceil(ceil(x / dx) / 2^r) (j2k_set_decode_area), equal to the
    reference's decode with that option."""
    a = SUB[tag]["variants"][vt]["args"]
    n = len(SUB[tag]["subsampling"])
    ref = _npz_planes(f"{GOLD}/{tag}.{vt}.dec.npz", n)
    cs = open(f"{GOLD}/{tag}.j2k", "rb").read()
    kw = {}
    if "-r" in a:
        kw["reduce"] = int(a[a.index("-r") + 1])
    if "-l" in a:
        kw["layers"] = int(a[a.index("-l") + 1])
    if "-d" in a:
        kw["window"] = tuple(int(v) for v in a[a.index("-d") + 1].split(","))
    d = codec.decompress(cs, **kw)
    cd = lambda v, s: -(-v // s)  # noqa: E731
    w, h = SUB[tag]["size"]
    args = SUB[tag]["args"]
    x0, y0 = (int(v) for v in args[args.index("-d") + 1].split(",")) if "-d" in args else (0, 0)
    R = 1 << kw.get("reduce", 0)
    for (dx, dy), x, r in zip(SUB[tag]["subsampling"], d, ref):
        if "window" in kw:
            assert x.shape == r.shape and np.array_equal(x, r)
        else:  # decoded samples: ceil(ceil(x1 / dx) / 2^r) - ceil(ceil(x0 / dx) / 2^r)
            assert_reduced_plane(x, r, cd(cd(y0 + h, dy), R) - cd(cd(y0, dy), R),
                                 cd(cd(x0 + w, dx), R) - cd(cd(x0, dx), R))


MARKER_VARIANTS = sorted((t, v) for t in MARKERS for v in MARKERS[t].get("variants", {}))


@pytest.mark.parametrize("tag,vt", MARKER_VARIANTS)
def test_decode_marker_fixture_options_match_reference(codec, tag, vt):
    """-r / -l over per-tile-component numres and packed headers, against the
    reference's decode with the same option."""
    a = MARKERS[tag]["variants"][vt]["args"]
    reduce = int(a[a.index("-r") + 1]) if "-r" in a else 0
    layers = int(a[a.index("-l") + 1]) if "-l" in a else 0
    ref = np.load(f"{GOLD}/{tag}.{vt}.dec.npy")
    d = codec.decompress(open(f"{GOLD}/{tag}.j2k", "rb").read(), reduce=reduce, layers=layers)
    assert d.shape == ref.shape
    assert int(np.abs(d.astype(np.int64) - ref).max()) == 0


def test_decode_mixed_cblksty_sorted(codec):
    """Components of different code-block styles (COC): the blocks go to one
    decode launch per style; with t1_dec_sort the work order is kept inside
    each style group.  Equal to the reference's decode either way."""
    import grokimagecompression_amd as grk
    cs = open(f"{GOLD}/mk_mixed_cblksty.j2k", "rb").read()
    ref = np.load(f"{GOLD}/mk_mixed_cblksty.dec.npy")
    for opts in ({}, {"t1_dec_sort": 1}, {"t1_dec_sort": 1, "t1_dec_bpw": 16}):
        with grk.dwt_options(**opts):
            assert np.array_equal(codec.decompress(cs), ref)
    ref = np.load(f"{GOLD}/mk_mixed_cblksty.r1.dec.npy")
    with grk.dwt_options(t1_dec_sort=1):
        assert np.array_equal(codec.decompress(cs, reduce=1), ref)


@pytest.mark.parametrize("tag", ["mk_tile_coc", "mk_ppt_tparts", "mk_main_coc", "mk_mixed_cblksty"])
def test_marker_fixtures_reduce_and_window(codec, tag):
    """The per-component / packed-header streams through -r 1 and a window:
    the window equals the crop of the full decode, and -r 1 equals a reduced
    decode of the same stream by the per-tile-component numres (every
    component of these keeps >= 2 resolutions)."""
    cs = open(f"{GOLD}/{tag}.j2k", "rb").read()
    full = codec.decompress(cs)
    h, w = full.shape[1:]
    x0, y0, x1, y1 = w // 5, h // 7, w - w // 4, h - h // 6
    win = codec.decompress(cs, window=(x0, y0, x1, y1))
    assert np.array_equal(win, full[:, y0:y1, x0:x1])
    red = codec.decompress(cs, reduce=1)
    assert red.shape == (full.shape[0], (h + 1) // 2, (w + 1) // 2)


VARIANTS = sorted((n, tag) for n in MAN for tag in MAN[n].get("variants", {}))


@pytest.mark.parametrize("name,tag", VARIANTS)
def test_decode_options_match_reference(codec, name, tag):
    """grk_decompress -l (layers) / -r (reduce) against the reference's own
    decode with those options (tests/golden/<case>.<tag>.dec.npy, written by
    oracle/make_golden.py from oracle/_ref): bit-exact, 9/7 included.  -l
    reproduces the reference's pass accounting (later layers' passes still
    count, T2.cpp:758-819)."""
    v = MAN[name]["variants"][tag]
    a = v["args"]
    reduce = int(a[a.index("-r") + 1]) if "-r" in a else 0
    layers = int(a[a.index("-l") + 1]) if "-l" in a else 0
    window = tuple(int(x) for x in a[a.index("-d") + 1].split(",")) if "-d" in a else None
    ref = np.load(f"{GOLD}/{name}.{tag}.dec.npy")
    d = codec.decompress(open(f"{GOLD}/{name}.j2k", "rb").read(), reduce=reduce, layers=layers, window=window)
    assert d.shape == ref.shape
    assert int(np.abs(d.astype(np.int64) - ref).max()) == 0


@pytest.mark.parametrize("name", ["g8_off35", "rgb12_I", "rgb8_128x96", "rgb12_tiles_I", "g16_I", "rgb8_nomct",
                                  "g8_off_tiles"])
def test_encode_fused_mct_dwt(codec, name):
    """Fused level 0 forced on (grkgpu_dwt_options.fuse_level0 = 1: the DC
    shift in the first DWT level's loads; MCT triples -- 9/7 included -- in
    one wavefront, k_dwt_fwd_mct3): same bytes as the reference."""
    import grokimagecompression_amd as grk
    with grk.dwt_options(fuse_level0=1):
        _encode_matches(codec, name)


def _encode_matches(codec, name):
    import grokimagecompression_amd as grk
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    assert codec.compress(img, bits, p, offset=off) == open(f"{GOLD}/{name}.j2k", "rb").read()


@pytest.mark.parametrize("name", ["rgb8_128x96", "rgb12_96x80", "rgb16_64", "rgb8_r10_tiles", "rgb8_uniform_64"])
def test_encode_unfused_rct(codec, name):
    """A 3-component 5/3 tile fuses the DC shift + RCT into DWT level 0 by
    default (k_dwt_fwd_mct3); fuse_level0 = 0 keeps the separate
    k_dcshift_mct_fwd pass, which must give the same bytes."""
    import grokimagecompression_amd as grk
    with grk.dwt_options(fuse_level0=0):
        _encode_matches(codec, name)


def test_device_resident_roundtrip(codec):
    import torch
    import grokimagecompression_amd as grk
    img = synth.synth_image(300, 411, 3, 10, 5)
    t = torch.from_numpy(img).cuda()
    for irrev in (False, True):
        b = codec.compress(t, 10, grk.CParams.make(irreversible=irrev))
        assert b == codec.compress(img, 10, grk.CParams.make(irreversible=irrev))
        out = codec.decompress(b, device_out=True)
        ref = codec.decompress(b)
        assert torch.equal(out.cpu(), torch.from_numpy(ref))
        if not irrev:
            assert np.array_equal(ref, img)


@pytest.mark.parametrize("irrev", [False, True, "f64"])
@pytest.mark.parametrize("shape_off", [((64, 64), (0, 0)), ((77, 100), (3, 5)), ((1, 37), (0, 1)),
                                       ((45, 1), (1, 0)), ((129, 200), (1, 1)), ((513, 257), (0, 3)),
                                       ((2, 3), (1, 1)), ((3, 130), (1, 0)), ((4, 5), (0, 1)), ((250, 121), (0, 0)),
                                       ((37, 260), (1, 1)), ((300, 497), (2, 2))])
@pytest.mark.parametrize("numres", [1, 2, 6, 9])
def test_dwt_stage_vs_oracle(oracle, irrev, shape_off, numres):
    """Per-level forward / inverse launches against the oracle; "f64": the
    9/7 forward lifting in f64 FMA + floor (f64_lift), at the magnitude of
    16-bit samples after the << 11 (2^26)."""
    import torch
    import grokimagecompression_amd as grk
    (h, w), (x0, y0) = shape_off
    f64 = irrev == "f64"
    irrev = bool(irrev)
    rng = np.random.default_rng(h * 1000 + w + numres)
    mag = (1 << 26) if f64 else (1 << 20) if irrev else 4096
    a = rng.integers(-mag, mag, size=(h, w)).astype(np.int32)
    ref = oracle.dwt_fwd(a, x0, y0, numres, irrev)
    t = torch.from_numpy(a).cuda()
    with grk.dwt_options(f64_lift=int(f64), f01_rows=0 if f64 else 4):
        grk.dwt_fwd(t, x0, y0, numres, irrev)
        torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), ref)
    # inverse: 5/3 on integers (exact reconstruction), 9/7 on floats
    if not irrev:
        grk.dwt_inv(t, x0, y0, numres, False)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), a)
    else:
        f = (rng.standard_normal((h, w)) * 100).astype(np.float32).view(np.int32)
        ref = oracle.dwt_inv(f, x0, y0, numres, True)
        t = torch.from_numpy(f.copy()).cuda()
        grk.dwt_inv(t, x0, y0, numres, True)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("irrev", [False, True])
@pytest.mark.parametrize("th", [16, 24])
def test_dwt_mid_th_vs_oracle(oracle, irrev, th):
    """Levels of 2^21 .. 2^23 samples in taller windows (mid_th = 16 / 24
    rows instead of 8), forward and inverse, against the oracle."""
    import torch
    import grokimagecompression_amd as grk
    h, w, x0, y0, numres = 1501, 1499, 1, 0, 4
    rng = np.random.default_rng(th + irrev)
    a = rng.integers(-(1 << 20), 1 << 20, size=(h, w)).astype(np.int32)
    with grk.dwt_options(mid_th=th):
        t = torch.from_numpy(a).cuda()
        grk.dwt_fwd(t, x0, y0, numres, irrev)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), oracle.dwt_fwd(a, x0, y0, numres, irrev))
        f = (rng.standard_normal((h, w)) * 100).astype(np.float32).view(np.int32) if irrev else \
            oracle.dwt_fwd(a, x0, y0, numres, False)
        ref = oracle.dwt_inv(f, x0, y0, numres, True) if irrev else a
        t = torch.from_numpy(f.copy()).cuda()
        grk.dwt_inv(t, x0, y0, numres, irrev)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("ny", ["2", "4", "6", "0", "mix", "g3", "d"])
@pytest.mark.parametrize("shape_off", [((32, 32), (0, 0)), ((33, 35), (1, 1)), ((77, 100), (3, 5)),
                                       ((129, 200), (1, 0)), ((513, 257), (0, 3)), ((300, 497), (2, 2)),
                                       ((37, 260), (1, 1)), ((700, 1030), (1, 1)), ((1100, 45), (0, 1))])
@pytest.mark.parametrize("numres", [3, 6])
def test_dwt_fused01_stage_vs_oracle(oracle, ny, shape_off, numres):
    """9/7 level pairs in one launch (k_dwt_fwd01, LL in LDS; default for
    pairs of >= 2^23 samples whose resolutions are >= 16 x 16, here forced
    onto every qualifying pair: 0+1, 2+3, ...), at each workgroup height
    (grkgpu_dwt_options.f01_rows = 2 / 4 / 6 level-0 row windows; 0 = two
    launches), on odd sizes and offsets (every cas parity, image edges inside
    the windows)."""
    import torch
    import grokimagecompression_amd as grk
    (h, w), (x0, y0) = shape_off
    rng = np.random.default_rng(h * 31 + w + numres)
    # "d" at the magnitude of 16-bit samples after the 9/7 << 11 (2^26)
    mag = 1 << (26 if ny == "d" else 20)
    a = rng.integers(-mag, mag, size=(h, w)).astype(np.int32)
    ref = oracle.dwt_fwd(a, x0, y0, numres, True)
    t = torch.from_numpy(a).cuda()
    # fuse every qualifying pair, not only chip-filling ones ("mix": pairs of
    # >= 2^16 samples with 4 row windows, smaller ones with 2)
    # "g3": workgroups walk groups of 3 columns top-down (pair_group)
    # "d": the f64 FMA + floor lifting (f64_lift)
    opts = dict(f01_rows=4, f01_min_samples=1 << 16, f01_small_min_samples=0) if ny == "mix" else \
        dict(f01_rows=4, f01_min_samples=0, pair_group=3) if ny == "g3" else \
        dict(f01_rows=4, f01_min_samples=0, f64_lift=1) if ny == "d" else dict(f01_rows=int(ny), f01_min_samples=0)
    with grk.dwt_options(pair_kernel=0, **opts):
        grk.dwt_fwd(t, x0, y0, numres, True)
        torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("irrev", [False, True])
@pytest.mark.parametrize("geo", [(0, 0), (0, 3), (14, 4), (8, 3), (30, 0), (62, 4), (16, 4)])
@pytest.mark.parametrize("shape_off", [((32, 32), (0, 0)), ((33, 35), (1, 1)), ((77, 100), (3, 5)),
                                       ((129, 200), (1, 0)), ((513, 257), (0, 3)), ((300, 497), (2, 2)),
                                       ((37, 260), (1, 1)), ((700, 1030), (1, 1)), ((1100, 45), (0, 1)),
                                       ((1081, 1921), (0, 1))])
@pytest.mark.parametrize("numres", [3, 6])
def test_dwt_pair_stage_vs_oracle(oracle, irrev, geo, shape_off, numres):
    """Forward level pairs streamed down column strips (k_dwt_fwd_pair, the
    default for pairs of >= 2^20 samples; here forced onto every qualifying
    pair: 0+1, 2+3, ...), 5/3 and 9/7, at several segment heights
    (pair_rows; 0 = by size) and 3 / 4 level-l wavefronts per workgroup
    (pair_waves; 0 = by width), on odd sizes and offsets: every cas parity,
    resolution edges inside the first / last chunk, strips and segments cut
    by the image edge."""
    import torch
    import grokimagecompression_amd as grk
    (h, w), (x0, y0) = shape_off
    rows, waves = geo
    if irrev and rows and rows % 8 != 6:
        rows += 6 - rows % 8 if rows % 8 < 6 else 14 - rows % 8  # the 9/7 stream's whole chunks (8k - 2)
    rng = np.random.default_rng(h * 31 + w + numres + 7 * irrev)
    a = rng.integers(-(1 << 20), 1 << 20, size=(h, w)).astype(np.int32) if irrev else \
        rng.integers(-(1 << 16), 1 << 16, size=(h, w)).astype(np.int32)
    ref = oracle.dwt_fwd(a, x0, y0, numres, irrev)
    t = torch.from_numpy(a).cuda()
    with grk.dwt_options(pair_kernel=2, f01_rows=4, pair_min_samples=0, pair_rows=rows, pair_waves=waves,
                         fuse_level0=0):
        grk.dwt_fwd(t, x0, y0, numres, irrev)
        torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("irrev", [False, True])
@pytest.mark.parametrize("fused", [0, 2, 4, "2g3"])
@pytest.mark.parametrize("shape_off", [((32, 32), (0, 0)), ((33, 35), (1, 1)), ((77, 100), (3, 5)),
                                       ((129, 200), (1, 0)), ((513, 257), (0, 3)), ((300, 497), (2, 2)),
                                       ((37, 260), (1, 1)), ((700, 1030), (1, 1)), ((1100, 45), (0, 1)),
                                       ((260, 37), (0, 0)), ((2160, 4096), (1, 0))])
@pytest.mark.parametrize("numres", [2, 3, 6])
def test_dwt_inv01_stage_vs_oracle(oracle, irrev, fused, shape_off, numres):
    """The two largest inverse levels in one launch (k_dwt_inv01: the smaller
    level's output in LDS; default when the larger has >= 2^23 samples), here
    forced onto every size (inv01_min_samples = 0) with 2 / 4 row windows of
    the smaller level per workgroup (0 = two launches), on odd
    sizes and offsets (every cas parity, image edges inside the windows):
    5/3 inverts the forward transform exactly, 9/7 (float, no FMA) equals the
    oracle's inverse bit for bit."""
    import torch
    import grokimagecompression_amd as grk
    (h, w), (x0, y0) = shape_off
    rng = np.random.default_rng(h * 7 + w + numres)
    opts = dict(inv01=2, pair_group=3) if fused == "2g3" else dict(inv01=fused)
    with grk.dwt_options(inv01_min_samples=0, **opts):
        if not irrev:
            a = rng.integers(-4096, 4096, size=(h, w)).astype(np.int32)
            t = torch.from_numpy(oracle.dwt_fwd(a, x0, y0, numres, False)).cuda()
            grk.dwt_inv(t, x0, y0, numres, False)
            torch.cuda.synchronize()
            assert np.array_equal(t.cpu().numpy(), a)
        else:
            f = (rng.standard_normal((h, w)) * 100).astype(np.float32).view(np.int32)
            ref = oracle.dwt_inv(f, x0, y0, numres, True)
            t = torch.from_numpy(f.copy()).cuda()
            grk.dwt_inv(t, x0, y0, numres, True)
            torch.cuda.synchronize()
            assert np.array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("irrev", [False, True])
def test_mct_stage_vs_oracle(oracle, irrev):
    import torch
    import grokimagecompression_amd as grk
    img = synth.synth_image(61, 129, 3, 12, 9)
    ref = oracle.dcshift_mct_fwd(list(img), [2048] * 3, 1, irrev)
    t = torch.from_numpy(img.copy()).cuda()
    grk.dcshift_mct_fwd(t, [2048] * 3, 1, irrev)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), np.stack(ref))


@pytest.mark.parametrize("name", ["C1_512_gray8", "C2_4k_rgb8", "C3_8k_rgb12_I", "C3_8k_rgb12", "C3_8k_rgb12_I_r20",
                                  "C5_dci4k_rgb12_cinema", "C5b_dci2k_rgb12_cinema",
                                  "C3_8k_rgb12_I_uniform", "C3_8k_rgb12_uniform", "C3_8k_rgb12_I_const",
                                  "C3_8k_rgb12_const"])
def test_large_config_hashes(codec, name):
    """BASELINE.json configs at full size: codestream sha256 == reference's,
    decoded-image sha256 == reference decoder's.  The C3 frame also as
    SURVEY 8(d)'s other inputs: uniform full-range 12-bit noise (the T1 worst
    case, every bit-plane of every block coded) and a constant frame."""
    import grokimagecompression_amd as grk
    import torch
    m = LARGE[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    t = torch.from_numpy(img).cuda()
    b = codec.compress(t, bits, p, offset=off)
    assert len(b) == m["j2k_len"]
    assert hashlib.sha256(b).hexdigest() == m["j2k_sha256"]
    d = codec.decompress(b)
    assert synth.image_sha256(d) == m["dec_sha256"]


@pytest.mark.parametrize("name", ["C3_8k_rgb12_I", "C3_8k_rgb12", "C3_8k_rgb12_I_uniform", "C3_8k_rgb12_uniform"])
def test_large_config_concurrent_calls(name):
    """The same full-size configs through calls that overlap on the GPU (two
    contexts on two threads): a call that is not alone takes the batch code
    paths -- 64 blocks per coder wavefront, the lane-per-block unstuff pass --
    and must give the reference's codestream and decoded image as well."""
    import threading
    import grokimagecompression_amd as grk
    import torch
    m = LARGE[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    t = torch.from_numpy(img).cuda()
    codecs = [grk.Codec(0), grk.Codec(0)]
    go = threading.Barrier(2)
    errs = []

    def run(c):
        try:
            go.wait()
            for _ in range(2):
                b = c.compress(t, bits, p, offset=off)
                assert hashlib.sha256(b).hexdigest() == m["j2k_sha256"]
                d = c.decompress(b)
                assert synth.image_sha256(d) == m["dec_sha256"]
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(c,)) for c in codecs]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for c in codecs:
        c.close()
    assert not errs, errs


def test_large_tiled_16k(codec):
    """C4: 16384^2 16-bit, 1024^2 tiles, 7 resolutions (256 tiles)."""
    import grokimagecompression_amd as grk
    import torch
    m = LARGE["C4_16k_gray16_tiled"]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    t = torch.from_numpy(img).cuda()
    del img
    b = codec.compress(t, bits, p, offset=off)
    assert hashlib.sha256(b).hexdigest() == m["j2k_sha256"]
    d = codec.decompress(b, device_out=True)
    assert torch.equal(d, t)


@pytest.mark.parametrize("name", sorted(n for n in MAN if oracle_supported(MAN[n]["args"])))
def test_reduced_decode_matches_oracle(codec, oracle, name):
    """grk_decompress -r: every reduce level of every golden codestream, GPU
    vs the oracle's reduced decode (bit-exact, 9/7 included).  The oracle's
    reduced decode is pinned for 5/3 by the forward-LL property
    (tests/test_oracle_golden.py::test_oracle_reduce_is_forward_ll); no
    reference fixture exists for -r."""
    import grokimagecompression_amd as grk
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    args = MAN[name]["args"]
    numres = int(args[args.index("-n") + 1]) if "-n" in args else 6
    for r in range(1, numres):
        ref = oracle.decode(gold, reduce=r)  # the decoded samples (no padding)
        d = codec.decompress(gold, reduce=r)
        h, w = ref.shape[1:]
        assert d.shape[0] == ref.shape[0] and h <= d.shape[1] <= h + 1 and w <= d.shape[2] <= w + 1, (name, r)
        assert np.array_equal(d[:, :h, :w], ref), (name, r)
        assert not d[:, h:].any() and not d[:, :, w:].any(), (name, r)
    with pytest.raises(grk.GrkGpuError):
        codec.decompress(gold, reduce=numres)


def test_reduced_decode_device_out_4k(codec):
    """Reduced decode of the 4K lossless config straight into HBM: the LL
    image equals the oracle's reduced decode."""
    import synth as sy
    import grokimagecompression_amd as grk
    img = sy.synth_image(2160, 3840, 3, 8, 2)
    b = codec.compress(img, 8, grk.CParams.make())
    d = codec.decompress(b, device_out=True, reduce=2)
    assert tuple(d.shape) == (3, 540, 960)
    import pyoracle
    assert np.array_equal(d.cpu().numpy(), pyoracle.decode(b, nthreads=8, reduce=2))


def _windows(x0, y0, x1, y1):
    w, h = x1 - x0, y1 - y0
    rng = np.random.default_rng(w * 7919 + h)
    wins = [(x0, y0, x1, y1), (x0, y0, x0 + 1, y0 + 1), (x1 - 1, y1 - 1, x1, y1),
            (x0 + w // 3, y0 + h // 3, x0 + (2 * w) // 3 + 1, y0 + (2 * h) // 3 + 1)]
    for _ in range(4):
        a = int(rng.integers(x0, x1))
        c = int(rng.integers(y0, y1))
        wins.append((a, c, int(rng.integers(a + 1, x1 + 1)), int(rng.integers(c + 1, y1 + 1))))
    return wins


@pytest.mark.parametrize("name", sorted(MAN))
def test_window_decode_matches_reference_crop(codec, name):
    """grk_set_decode_area: the window decode of every golden codestream
    equals the REFERENCE decoder's full output cropped to the window (pinned
    by the reference fixtures), for full, 1-sample, corner, centre and random
    windows (9/7, offsets, multi-tile included)."""
    import grokimagecompression_amd as grk
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    ref = np.load(f"{GOLD}/{name}.dec.npy")
    hd = grk.read_header(gold)
    for win in _windows(hd.x0, hd.y0, hd.x1, hd.y1):
        x0, y0, x1, y1 = win
        d = codec.decompress(gold, window=win)
        exp = ref[:, y0 - hd.y0:y1 - hd.y0, x0 - hd.x0:x1 - hd.x0]
        assert d.shape == exp.shape, (name, win)
        assert np.array_equal(d, exp), (name, win)
    with pytest.raises(grk.GrkGpuError):
        codec.decompress(gold, window=(hd.x1, hd.y1, hd.x1 + 5, hd.y1 + 5))


def test_window_decode_16k_tiles(codec):
    """A window across four 1024^2 tiles of the 16K config decodes only those
    tiles and equals the full decode's crop."""
    import torch
    import grokimagecompression_amd as grk
    m = LARGE["C4_16k_gray16_tiled"]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    b = codec.compress(img, bits, p, offset=off)
    win = (1000, 3000, 1100, 3100)
    d = codec.decompress(b, window=win, device_out=True)
    assert torch.equal(d.cpu(), torch.from_numpy(img[:, 3000:3100, 1000:1100].copy()))


@pytest.mark.parametrize("hw", [(1024, 1536), (1536, 2048), (1100, 1700)])
@pytest.mark.parametrize("irrev", [False, True])
def test_mid_size_blocks_per_wave(codec, oracle, hw, irrev):
    """Images of 1,000-4,000 code-blocks: the T1 lane coders run 2-32 blocks
    per wavefront there (kernels.hip t1_blocks_per_wave; the goldens have
    fewer than 1,024 blocks -- one per wavefront -- and the full-size configs
    more than 4,096 -- 64).  Codestream == the oracle's, decode == the
    oracle's decode."""
    import grokimagecompression_amd as grk
    h, w = hw
    img = synth.synth_image(h, w, 3, 10, h + w)
    b = codec.compress(img, 10, grk.CParams.make(irreversible=irrev))
    ref = oracle.encode(img, 10, oracle.params(irreversible=irrev, nthreads=8))
    assert b == ref
    d = codec.decompress(b)
    assert np.array_equal(d, oracle.decode(ref, nthreads=8))


@pytest.mark.parametrize("name,dtype", [("rgb8_128x96", "uint8"), ("rgb8_128x96", "uint16"), ("rgb12_I", "uint16"),
                                        ("rgb12_96x80", "uint16"), ("g8_off35", "uint8"), ("g16_I", "uint16"),
                                        ("rgb8_r10_tiles", "uint8"), ("g8_off_tiles", "uint16"),
                                        ("rgb16_64", "uint16")])
def test_encode_sample_formats(codec, name, dtype):
    """Image planes handed over at the image file's sample width
    (grkgpu_compress_ex, GRKGPU_SAMPLE_U8 / U16: host, pinned host and
    device tensors), widened to int32 on the GPU in the DC shift + MCT pass or
    the fused DWT level 0: the reference's bytes."""
    import torch
    import grokimagecompression_amd as grk
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    a = img.astype(dtype)
    assert codec.compress(a, bits, p, offset=off) == gold
    t = torch.from_numpy(a)
    assert codec.compress(t.pin_memory(), bits, p, offset=off) == gold
    assert codec.compress(t.cuda(), bits, p, offset=off) == gold
    # an odd-width view of the planes (no pair loads) still matches
    if a.shape[2] > 2:
        sub = np.ascontiguousarray(a[:, :, 1:])
        assert codec.compress(sub, bits, p, offset=off) == codec.compress(sub.astype(np.int32), bits, p, offset=off)


@pytest.mark.parametrize("bits,irrev", [(12, False), (12, True), (8, False), (16, True)])
def test_encode_signed_sample_formats(codec, bits, irrev):
    """Signed components as int8 / int16 samples (GRKGPU_SAMPLE_I8 / I16):
    the same codestream as their int32 planes.  A format that cannot hold the
    component (unsigned samples for a signed image, 8-bit samples of a 12-bit
    image) is refused by the C ABI; the Python layer widens such numpy / torch
    samples to int32 first, so they encode exactly as their int32 planes."""
    import ctypes
    import torch
    import grokimagecompression_amd as grk
    rng = np.random.default_rng(bits)
    img = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), size=(3, 70, 93)).astype(np.int32)
    p = grk.CParams.make(irreversible=irrev)
    ref = codec.compress(img, bits, p, sgnd=True)
    small = np.int8 if bits <= 8 else np.int16
    assert codec.compress(img.astype(small), bits, p, sgnd=True) == ref
    mism = [((np.abs(img) % (1 << (bits - 1))).astype(np.uint16), True)]  # in range, unsigned storage
    if bits > 8:
        mism.append(((img + (1 << (bits - 1))).astype(np.uint8), False))
    for a, sg in mism:
        wide = codec.compress(a.astype(np.int32), bits, p, sgnd=sg)
        assert codec.compress(a, bits, p, sgnd=sg) == wide
        if a.dtype == np.uint8:  # torch has no uint16 before 2.3: checked on uint8
            assert codec.compress(torch.from_numpy(a).cuda(), bits, p, sgnd=sg) == wide
        # the ABI refuses the format itself
        d, pl, keep = codec._image(a.astype(np.int32), bits, (0, 0), sg)
        pl.sample_fmt = grk.SAMPLE_U16 if a.dtype == np.uint16 else grk.SAMPLE_U8
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        assert grk.lib().grkgpu_compress_ex(codec._ctx, ctypes.byref(d), ctypes.byref(p), ctypes.byref(pl), 0,
                                            0xFFFFFFFF, grk.PART_ALL, ctypes.byref(out), ctypes.byref(n)) != 0
