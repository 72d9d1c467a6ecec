"""ctypes binding of the CPU oracle (oracle/build/libgrk_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libgrk_oracle.so")
MAXC = 16


class OrcImage(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_uint32), ("y0", ctypes.c_uint32), ("x1", ctypes.c_uint32), ("y1", ctypes.c_uint32),
                ("numcomps", ctypes.c_uint32), ("prec", ctypes.c_uint32 * MAXC), ("sgnd", ctypes.c_int32 * MAXC),
                ("data", ctypes.POINTER(ctypes.c_int32) * MAXC)]


class OrcParams(ctypes.Structure):
    _fields_ = [("numres", ctypes.c_uint32), ("cblkw", ctypes.c_uint32), ("cblkh", ctypes.c_uint32),
                ("irreversible", ctypes.c_int32), ("mct", ctypes.c_int32), ("tile_on", ctypes.c_int32),
                ("tdx", ctypes.c_uint32), ("tdy", ctypes.c_uint32), ("tx0", ctypes.c_uint32), ("ty0", ctypes.c_uint32),
                ("nthreads", ctypes.c_int32)]


class OrcPass(ctypes.Structure):
    _fields_ = [("rate", ctypes.c_uint32), ("len", ctypes.c_uint32), ("term", ctypes.c_uint32)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.orc_encode.argtypes = [ctypes.POINTER(OrcImage), ctypes.POINTER(OrcParams),
                                    ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_size_t)]
        _lib.orc_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(OrcImage), ctypes.c_int32]
        _lib.orc_decode_reduce.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(OrcImage), ctypes.c_int32,
                                           ctypes.c_uint32]
        _lib.orc_free.argtypes = [ctypes.c_void_p]
        _lib.orc_image_free.argtypes = [ctypes.POINTER(OrcImage)]
        _lib.orc_dwt_fwd.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 5 + [ctypes.c_int32, ctypes.c_int32]
        _lib.orc_dwt_inv.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 5 + [ctypes.c_int32, ctypes.c_int32]
        _lib.orc_dcshift_mct_fwd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        _lib.orc_t1_encode_cblk.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                            ctypes.c_uint32, ctypes.POINTER(OrcPass), ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(ctypes.c_uint32)]
        _lib.orc_t1_encode_cblk_nmse.argtypes = _lib.orc_t1_encode_cblk.argtypes + [ctypes.c_void_p]
        _lib.orc_t1_wmsedec.restype = ctypes.c_double
        _lib.orc_t1_wmsedec.argtypes = [ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_int32, ctypes.c_uint32, ctypes.c_double, ctypes.c_void_p,
                                        ctypes.c_uint32]
        _lib.orc_t1_decode_cblk.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        _lib.orc_count_cblks.argtypes = [ctypes.c_uint32] * 7
        _lib.orc_count_cblks.restype = ctypes.c_uint32
    return _lib


def params(numres=6, cblk=(64, 64), irreversible=False, mct=-1, tiles=None, tile_offset=(0, 0), nthreads=0):
    p = OrcParams()
    p.numres = numres
    p.cblkw = int(np.log2(cblk[0]))
    p.cblkh = int(np.log2(cblk[1]))
    p.irreversible = 1 if irreversible else 0
    p.mct = mct
    if tiles:
        p.tile_on = 1
        p.tdx, p.tdy = tiles
        p.tx0, p.ty0 = tile_offset
    p.nthreads = nthreads
    return p


def params_from_args(args, nthreads=0):
    """Map the grk_compress options used by the golden cases to OrcParams."""
    kw = {}
    i = 0
    while i < len(args):
        a = args[i]
        if a == "-I":
            kw["irreversible"] = True
        elif a == "-n":
            kw["numres"] = int(args[i + 1]); i += 1
        elif a == "-b":
            w, h = args[i + 1].split(","); kw["cblk"] = (int(w), int(h)); i += 1
        elif a == "-t":
            w, h = args[i + 1].split(","); kw["tiles"] = (int(w), int(h)); i += 1
        elif a == "-T":
            x, y = args[i + 1].split(","); kw["tile_offset"] = (int(x), int(y)); i += 1
        elif a == "-Y":
            kw["mct"] = int(args[i + 1]); i += 1
        elif a == "-d":
            i += 1  # image offset handled by the caller
        else:
            raise ValueError(a)
        i += 1
    return params(nthreads=nthreads, **kw)


def image_offset_from_args(args):
    if "-d" in args:
        x, y = args[args.index("-d") + 1].split(",")
        return int(x), int(y)
    return 0, 0


def encode(img, prec, p, offset=(0, 0), sgnd=False):
    """img: (c,h,w) int32 -> bytes"""
    img = np.ascontiguousarray(img, dtype=np.int32)
    c, h, w = img.shape
    oi = OrcImage()
    oi.x0, oi.y0 = offset
    oi.x1, oi.y1 = offset[0] + w, offset[1] + h
    oi.numcomps = c
    for k in range(c):
        oi.prec[k] = prec
        oi.sgnd[k] = 1 if sgnd else 0
        oi.data[k] = img[k].ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    rc = lib().orc_encode(ctypes.byref(oi), ctypes.byref(p), ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError("orc_encode failed %d" % rc)
    b = ctypes.string_at(out, n.value)
    lib().orc_free(out)
    return b


def decode(buf, nthreads=0, reduce=0):
    """bytes -> (c,h,w) int32; reduce > 0: the image at resolution numres-1-reduce"""
    oi = OrcImage()
    src = ctypes.create_string_buffer(bytes(buf), len(buf))
    rc = lib().orc_decode_reduce(src, len(buf), ctypes.byref(oi), nthreads, reduce)
    if rc != 0:
        raise RuntimeError("orc_decode failed %d" % rc)
    w, h = oi.x1 - oi.x0, oi.y1 - oi.y0
    out = np.empty((oi.numcomps, h, w), dtype=np.int32)
    for k in range(oi.numcomps):
        out[k] = np.ctypeslib.as_array(oi.data[k], shape=(h * w,)).reshape(h, w)
    lib().orc_image_free(ctypes.byref(oi))
    return out


def dwt_fwd(buf, x0, y0, numres, irreversible, nthreads=0):
    a = np.ascontiguousarray(buf, dtype=np.int32).copy()
    h, w = a.shape
    lib().orc_dwt_fwd(a.ctypes.data, x0, y0, x0 + w, y0 + h, numres, 1 if irreversible else 0, nthreads)
    return a


def dwt_inv(buf, x0, y0, numres, irreversible, nthreads=0):
    a = np.ascontiguousarray(buf).copy()
    h, w = a.shape
    lib().orc_dwt_inv(a.ctypes.data, x0, y0, x0 + w, y0 + h, numres, 1 if irreversible else 0, nthreads)
    return a


def dcshift_mct_fwd(planes, shifts, mct, irreversible):
    p = [np.ascontiguousarray(x, dtype=np.int32).copy() for x in planes]
    n = p[0].size
    sh = np.asarray(shifts, dtype=np.int32)
    ptrs = [x.ctypes.data for x in p] + [None] * (3 - len(p))
    lib().orc_dcshift_mct_fwd(ptrs[0], ptrs[1], ptrs[2], len(p), n, sh.ctypes.data, mct, 1 if irreversible else 0)
    return p


def t1_encode_cblk(block, orient, qmfbid, inv_step=0, nmse=False):
    """T1 encode of one block (preEncode quantisation included): (bytes,
    [(rate, len, term)] per pass, numbps) -- plus, with nmse=True, the
    per-pass normalised distortion decrease sums (t1.cpp nmsedec)."""
    blk = np.ascontiguousarray(block, dtype=np.int32)
    h, w = blk.shape
    cap = w * h * 8 + 64
    out = (ctypes.c_uint8 * (cap + 1))()
    passes = (OrcPass * 100)()
    nbps = ctypes.c_uint32()
    olen = ctypes.c_uint32()
    nm = (ctypes.c_int32 * 100)()
    n = lib().orc_t1_encode_cblk_nmse(blk.ctypes.data, w, w, h, orient, qmfbid, inv_step,
                                      ctypes.addressof(out) + 1, cap, passes, ctypes.byref(nbps), ctypes.byref(olen),
                                      nm)
    data = bytes(out)[1:1 + olen.value]
    res = (data, [(passes[i].rate, passes[i].len, passes[i].term) for i in range(n)], nbps.value)
    return res + ([nm[i] for i in range(n)],) if nmse else res


def t1_wmsedec(nmsedec, compno, level, orient, bpno, qmfbid, stepsize, mct_norms=None):
    """t1_getwmsedec (t1.cpp:912-930) of one pass."""
    norms = (ctypes.c_double * 3)(*mct_norms) if mct_norms else None
    return lib().orc_t1_wmsedec(nmsedec, compno, level, orient, bpno, qmfbid, stepsize, norms,
                                len(mct_norms) if mct_norms else 0)


def t1_decode_cblk(data, numpasses, numbps, w, h, orient):
    buf = ctypes.create_string_buffer(bytes(data) + b"\0\0", len(data) + 2)
    out = np.zeros((h, w), dtype=np.int32)
    lib().orc_t1_decode_cblk(buf, len(data), numpasses, numbps, w, h, orient, out.ctypes.data)
    return out
