"""Per-stage C-ABI entry points against the oracle (INTEGRATION.md §2's
"per-stage route"): grkgpu_t1_encode_blocks, grkgpu_t1_decode_blocks and
grkgpu_mct_inv_dcshift, on device buffers, bit-exact.

  * T1 encode: the oracle's t1_encode_cblk (restating t1.cpp t1_encode_cblk,
    :1160-1326) on the same quantised blocks -- numbps, pass count, every
    cumulative pass rate and the MQ bytes; with_distortion=1 must not change
    them, and its per-pass distortion sums equal the oracle's restatement
    exactly (the weighted, cumulative values are checked against the
    reference host's own T1 in tests/test_gpu_plugin.py's debug-state run).
  * T1 decode: the oracle's t1_decode_cblk (t1.cpp:1038-1130) + the
    whole-tile post_decode scaling (T1Part1.cpp:216-330; 5/3: v/2, 9/7:
    float(v) * step), for all passes and for truncated pass counts (a layer
    cut), through the product's v5 decoder.
  * inverse MCT + DC shift + clamp: RCT round trip against the oracle's
    forward transform, and ICT against a float32 restatement of
    mct.cpp decode_irrev (:352-408: separate mul / add, round to nearest
    even) with the DC shift and clamp of TileProcessor.cpp:1303-1432.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ENC_RESULT = np.dtype([("numbps", "<u4"), ("numpasses", "<u4"), ("len", "<u4"), ("pad", "<u4"),
                       ("nsym", "<u4"), ("p1", "<u4"), ("p2", "<u4"), ("p3", "<u4"),
                       ("rate", "<u4", 96), ("nmsedec", "<i4", 96)])
ENC_BLOCK = np.dtype([("coef_off", "<u8"), ("out_off", "<u8"), ("stride", "<u4"), ("w", "<u4"), ("h", "<u4"),
                      ("orient", "<u4"), ("qmfbid", "<i4"), ("inv_step", "<i4")])
DEC_BLOCK = np.dtype([("data_off", "<u8"), ("dst_off", "<u8"), ("len", "<u4"), ("numpasses", "<u4"),
                      ("numbps", "<u4"), ("w", "<u4"), ("h", "<u4"), ("orient", "<u4"), ("dstride", "<u4"),
                      ("irrev", "<i4"), ("step", "<f4"), ("pad", "<u4")])
MAX_SEG = 64 * 64 * 4 + 64
SHAPES = [(64, 64), (32, 32), (64, 16), (16, 64), (7, 3), (1, 1), (1, 64), (64, 1), (33, 47), (4, 4)]


def _blocks(seed):
    """(h, w, orient, qmfbid, inv_step, block) cases: Laplacian-ish values with
    smooth structure, an all-zero block and a single-sample spike."""
    rng = np.random.default_rng(seed)
    out = []
    for i, (h, w) in enumerate(SHAPES):
        for qmfbid, inv in ((1, 0), (0, 6553), (0, 1111)):
            orient = (i + qmfbid) % 4
            yy, xx = np.mgrid[0:h, 0:w]
            base = (200 * np.sin(xx / 5.0 + i) * np.cos(yy / 7.0)).astype(np.int64)
            noise = rng.laplace(0, 30 + 20 * i, size=(h, w)).astype(np.int64)
            v = base + noise
            if qmfbid == 0:
                v = v << 8  # 9/7 coefficients carry fixed-point fraction bits
            out.append((h, w, orient, qmfbid, inv, v.astype(np.int32)))
    out.append((64, 64, 0, 1, 0, np.zeros((64, 64), np.int32)))
    spike = np.zeros((17, 9), np.int32)
    spike[8, 4] = -1234
    out.append((17, 9, 3, 1, 0, spike))
    return out


def _gpu_encode(cases, with_distortion):
    import torch
    import grokimagecompression_amd as grk
    L = grk.lib()
    n = len(cases)
    coef = np.concatenate([c[5].ravel() for c in cases]).astype(np.int32)
    eb = np.zeros(n, ENC_BLOCK)
    off = 0
    for i, (h, w, orient, qmfbid, inv, blk) in enumerate(cases):
        eb[i] = (off, 16 + i * (MAX_SEG + 16), w, w, h, orient, qmfbid, inv)
        off += h * w
    dev = torch.device("cuda", 0)
    t_coef = torch.from_numpy(coef).to(dev)
    t_blocks = torch.from_numpy(eb.view(np.uint8)).to(dev)
    t_out = torch.zeros(16 + n * (MAX_SEG + 16), dtype=torch.uint8, device=dev)
    t_res = torch.zeros(n * ENC_RESULT.itemsize, dtype=torch.uint8, device=dev)
    t_scr = torch.empty(L.grkgpu_t1_scratch_bytes_n(n) + 256, dtype=torch.uint8, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(0).cuda_stream)
    grk._check(L.grkgpu_t1_encode_blocks(t_blocks.data_ptr(), n, t_coef.data_ptr(), t_scr.data_ptr(),
                                         t_out.data_ptr(), t_res.data_ptr(), with_distortion, s))
    torch.cuda.synchronize()
    res = t_res.cpu().numpy().view(ENC_RESULT)
    out = t_out.cpu().numpy()
    return res, out, eb


@pytest.mark.parametrize("seed", [1, 2])
def test_t1_encode_blocks_vs_oracle(oracle, seed):
    cases = _blocks(seed)
    res, out, eb = _gpu_encode(cases, 0)
    for i, (h, w, orient, qmfbid, inv, blk) in enumerate(cases):
        data, passes, nbps = oracle.t1_encode_cblk(blk, orient, qmfbid, inv)
        r = res[i]
        assert r["numbps"] == nbps, i
        assert r["numpasses"] == len(passes), i
        assert list(r["rate"][:len(passes)]) == [p[0] for p in passes], i
        o = int(eb[i]["out_off"])
        assert bytes(out[o:o + len(data)]) == data, i


@pytest.mark.parametrize("seed", [3, 5])
def test_t1_encode_blocks_distortion(oracle, seed):
    """with_distortion=1: the bytes and rates are unchanged, and every pass's
    normalised distortion decrease sum (t1_encode_cblk's nmsedec, the input
    of t1_getwmsedec, t1.cpp:912-930 / :1249-1254) equals the oracle's
    restatement exactly (oracle/grk_oracle.c orc_t1_encode_cblk_nmse: the
    t1_generate_luts.cpp:290-318 tables, accumulated at t1.cpp:217 / :452 /
    :684)."""
    cases = _blocks(seed)
    r0, o0, _ = _gpu_encode(cases, 0)
    r1, o1, _ = _gpu_encode(cases, 1)
    assert np.array_equal(o0, o1)
    for i, (h, w, orient, qmfbid, inv, blk) in enumerate(cases):
        np_ = int(r1[i]["numpasses"])
        assert list(r1[i]["rate"][:np_]) == list(r0[i]["rate"][:np_])
        _, passes, nbps, nm = oracle.t1_encode_cblk(blk, orient, qmfbid, inv, nmse=True)
        assert np_ == len(passes), i
        assert [int(v) for v in r1[i]["nmsedec"][:np_]] == nm, i


def _gpu_decode(items):
    """items: (data, numpasses, numbps, w, h, orient, irrev, step) -> list of (h,w) int32."""
    import torch
    import grokimagecompression_amd as grk
    L = grk.lib()
    n = len(items)
    blob = bytearray(16)
    db = np.zeros(n, DEC_BLOCK)
    dst_off = 0
    for i, (data, npass, nbps, w, h, orient, irrev, step) in enumerate(items):
        db[i] = (len(blob), dst_off, len(data), npass, nbps, w, h, orient, w, irrev, step, 0)
        blob += data + bytes(16)
        dst_off += w * h
    dev = torch.device("cuda", 0)
    t_data = torch.from_numpy(np.frombuffer(bytes(blob) + bytes(64), np.uint8).copy()).to(dev)
    t_blocks = torch.from_numpy(db.view(np.uint8)).to(dev)
    t_dst = torch.full((dst_off + 16,), 0x5A5A5A5A, dtype=torch.int32, device=dev)
    assert L.grkgpu_t1_scratch_bytes_n(n) == (n + 63) // 64 * 64 * L.grkgpu_t1_scratch_bytes()  # whole 64-block groups
    t_scr = torch.empty(L.grkgpu_t1_scratch_bytes_n(n) + 256, dtype=torch.uint8, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(0).cuda_stream)
    grk._check(L.grkgpu_t1_decode_blocks(t_blocks.data_ptr(), n, t_data.data_ptr(), t_scr.data_ptr(),
                                         t_dst.data_ptr(), s))
    torch.cuda.synchronize()
    d = t_dst.cpu().numpy()
    outs = []
    for i in range(n):
        w, h = int(db[i]["w"]), int(db[i]["h"])
        o = int(db[i]["dst_off"])
        outs.append(d[o:o + w * h].reshape(h, w))
    return outs


def _post(v, irrev, step):
    if not irrev:
        return (np.trunc(v / 2)).astype(np.int32)  # C integer division
    return (v.astype(np.float32) * np.float32(step)).view(np.int32)


@pytest.mark.parametrize("seed", [4])
def test_t1_decode_blocks_vs_oracle(oracle, seed):
    items, refs = [], []
    for (h, w, orient, qmfbid, inv, blk) in _blocks(seed):
        data, passes, nbps = oracle.t1_encode_cblk(blk, orient, qmfbid, inv)
        if not passes:
            continue
        irrev = 1 if qmfbid == 0 else 0
        step = 0.0 if not irrev else 1.0 / (inv / 8192.0) / 4.0
        for npass in sorted({len(passes), max(1, len(passes) // 2), 1}):
            rate = passes[npass - 1][0]
            seg = data[:rate]
            items.append((seg, npass, nbps, w, h, orient, irrev, step))
            ref = oracle.t1_decode_cblk(seg, npass, nbps, w, h, orient)
            refs.append(_post(ref, irrev, step))
    outs = _gpu_decode(items)
    for i, (o, r) in enumerate(zip(outs, refs)):
        assert np.array_equal(o, r), (i, items[i][1:6])


def _ict_inv_ref(yuv, prec):
    y, u, v = [p.view(np.float32) for p in yuv]
    f = np.float32
    r = y + v * f(1.402)
    g = (y - u * f(0.34413)) - v * f(0.71414)
    b = y + u * f(1.772)
    out = [np.rint(c).astype(np.int32) + (1 << (prec - 1)) for c in (r, g, b)]
    return [np.clip(c, 0, (1 << prec) - 1) for c in out]


@pytest.mark.parametrize("prec", [8, 12])
def test_mct_inv_dcshift(oracle, prec):
    import torch
    import grokimagecompression_amd as grk
    import synth
    img = synth.synth_image(37, 53, 3, prec, 9)
    shift = 1 << (prec - 1)
    # RCT: forward (oracle) then the GPU inverse restores the image exactly
    fwd = oracle.dcshift_mct_fwd(list(img), [shift] * 3, 1, False)
    t = torch.from_numpy(np.stack(fwd)).cuda()
    grk.mct_inv_dcshift(t, prec, False, 1, False)
    assert np.array_equal(t.cpu().numpy(), img)
    # ICT: float planes (as the inverse 9/7 DWT leaves them) vs the restatement
    rng = np.random.default_rng(prec)
    yuv = [(rng.standard_normal((37, 53)) * (1 << (prec - 2))).astype(np.float32) for _ in range(3)]
    yuv[0] += np.float32(0.37)  # fractions on the rounding boundary side
    raw = [p.view(np.int32) for p in yuv]
    t = torch.from_numpy(np.stack(raw)).cuda()
    grk.mct_inv_dcshift(t, prec, False, 1, True)
    ref = _ict_inv_ref(raw, prec)
    assert np.array_equal(t.cpu().numpy(), np.stack(ref))
    # no MCT: DC shift + clamp only (values past the range clamp)
    planes = rng.integers(-(1 << prec), 1 << prec, size=(2, 20, 30)).astype(np.int32)
    t = torch.from_numpy(planes.copy()).cuda()
    grk.mct_inv_dcshift(t, prec, False, 0, False)
    assert np.array_equal(t.cpu().numpy(), np.clip(planes + shift, 0, (1 << prec) - 1))
