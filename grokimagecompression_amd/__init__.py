"""grokimagecompression_amd -- MI355X-native JPEG 2000 hot path, Grok-compatible.

Python host mirror of the reference's compress / decompress entry points
(grk_compress / grk_decompress, Grok v5.1.0) over the C ABI in
include/grk_mi355x.h (libgrk_mi355x.so, built in-tree under lib/).

    import grokimagecompression_amd as grk
    codec = grk.Codec(device=0)
    j2k = codec.compress(img, prec=8)                 # img: (c,h,w) int32 numpy or torch.cuda tensor
    out = codec.decompress(j2k)                       # numpy (c,h,w) int32
    out = codec.decompress(j2k, device_out=True)      # torch.cuda tensor

The product path never falls back to the CPU: if the extension is missing or
no gfx950 device is present, every entry point raises GrkGpuError.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GRKGPU_LIB: another build of the library (A/B experiments)
LIB_PATH = os.environ.get("GRKGPU_LIB") or os.path.join(_HERE, "lib", "libgrk_mi355x.so")
MAXC = 16

__all__ = ["Codec", "CParams", "GrkGpuError", "lib", "build", "read_header"]


class GrkGpuError(RuntimeError):
    pass


class ImageDesc(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_uint32), ("y0", ctypes.c_uint32), ("x1", ctypes.c_uint32), ("y1", ctypes.c_uint32),
                ("numcomps", ctypes.c_uint32), ("prec", ctypes.c_uint32 * MAXC), ("sgnd", ctypes.c_int32 * MAXC),
                ("dx", ctypes.c_uint32 * MAXC), ("dy", ctypes.c_uint32 * MAXC)]


class DParams(ctypes.Structure):
    """grkgpu_dparams (grk_dparameters subset, grok.h:694-735)."""
    _fields_ = [("cp_reduce", ctypes.c_uint32), ("cp_layer", ctypes.c_uint32), ("DA_x0", ctypes.c_uint32),
                ("DA_y0", ctypes.c_uint32), ("DA_x1", ctypes.c_uint32), ("DA_y1", ctypes.c_uint32)]


class Poc(ctypes.Structure):
    """grk_poc (grok.h:393-410): grk_compress -P T<tile>=r0,c0,l1,r1,c1,PROG."""
    _fields_ = [("tile", ctypes.c_uint32), ("resno0", ctypes.c_uint32), ("compno0", ctypes.c_uint32),
                ("layno1", ctypes.c_uint32), ("resno1", ctypes.c_uint32), ("compno1", ctypes.c_uint32),
                ("prog", ctypes.c_int32)]


PROGS = {"LRCP": 0, "RLCP": 1, "RPCL": 2, "PCRL": 3, "CPRL": 4}
CSTY_PRT, CSTY_SOP, CSTY_EPH = 1, 2, 4
PROFILE_CINEMA_2K, PROFILE_CINEMA_4K = 3, 4


class CParams(ctypes.Structure):
    """grk_cparameters subset (grok.h:447-570), mirrored by include/grk_mi355x.h."""
    _fields_ = [("numresolution", ctypes.c_uint32), ("cblockw_init", ctypes.c_uint32),
                ("cblockh_init", ctypes.c_uint32), ("irreversible", ctypes.c_int32), ("tcp_mct", ctypes.c_int32),
                ("tile_size_on", ctypes.c_int32), ("cp_tdx", ctypes.c_uint32), ("cp_tdy", ctypes.c_uint32),
                ("cp_tx0", ctypes.c_uint32), ("cp_ty0", ctypes.c_uint32),
                ("tcp_numlayers", ctypes.c_uint32), ("tcp_rates", ctypes.c_double * 100),
                ("tcp_distoratio", ctypes.c_double * 100), ("cp_disto_alloc", ctypes.c_int32),
                ("cp_fixed_quality", ctypes.c_int32), ("rate_control_algorithm", ctypes.c_int32),
                ("csty", ctypes.c_uint32), ("res_spec", ctypes.c_uint32), ("prcw_init", ctypes.c_uint32 * 33),
                ("prch_init", ctypes.c_uint32 * 33), ("prog_order", ctypes.c_int32), ("numpocs", ctypes.c_uint32),
                ("POC", Poc * 32), ("tp_on", ctypes.c_int32), ("tp_flag", ctypes.c_int32), ("rsiz", ctypes.c_uint32),
                ("framerate", ctypes.c_uint32), ("max_cs_size", ctypes.c_uint64), ("max_comp_size", ctypes.c_uint64),
                ("cblk_sty", ctypes.c_uint32), ("roi_compno", ctypes.c_int32), ("roi_shift", ctypes.c_uint32),
                ("pad_", ctypes.c_uint32), ("mct_ncomp", ctypes.c_uint32), ("mct_matrix", ctypes.c_float * (MAXC * MAXC)),
                ("mct_dc_shift", ctypes.c_int32 * MAXC)]

    def set_mct(self, matrix, dc_shift):
        """grk_set_MCT: a custom array-based MCT (grkgpu_set_mct)."""
        n = len(dc_shift)
        m = (ctypes.c_float * (n * n))(*[float(v) for v in np.asarray(matrix, dtype=np.float32).ravel()])
        s = (ctypes.c_int32 * n)(*[int(v) for v in dc_shift])
        _check(lib().grkgpu_set_mct(ctypes.byref(self), m, s, n))
        return self

    @classmethod
    def make(cls, numresolution=6, cblk=(64, 64), irreversible=False, mct=-1, tiles=None, tile_offset=(0, 0)):
        p = cls()
        lib().grkgpu_default_cparams(ctypes.byref(p))
        p.numresolution = numresolution
        p.cblockw_init, p.cblockh_init = cblk
        p.irreversible = 1 if irreversible else 0
        p.tcp_mct = mct
        if tiles:
            p.tile_size_on = 1
            p.cp_tdx, p.cp_tdy = tiles
        p.cp_tx0, p.cp_ty0 = tile_offset
        return p

    @classmethod
    def from_cli(cls, args):
        """Map grk_compress command-line options to params (the option
        handling of grk_compress.cpp:564-1620); returns (params, image_offset)."""
        p = cls.make()
        off, i = (0, 0), 0
        cinema = 0
        while i < len(args):
            a = args[i]
            v = args[i + 1] if i + 1 < len(args) else ""
            if a == "-I":
                p.irreversible = 1
            elif a in ("-S", "-SOP"):
                p.csty |= CSTY_SOP
            elif a in ("-E", "-EPH"):
                p.csty |= CSTY_EPH
            else:
                i += 1
                if a == "-n":
                    p.numresolution = int(v)
                elif a == "-b":
                    p.cblockw_init, p.cblockh_init = (int(x) for x in v.split(","))
                elif a == "-t":
                    p.tile_size_on = 1
                    p.cp_tdx, p.cp_tdy = (int(x) for x in v.split(","))
                elif a == "-T":
                    p.cp_tx0, p.cp_ty0 = (int(x) for x in v.split(","))
                elif a == "-Y":
                    p.tcp_mct = int(v)
                elif a == "-mct":  # oracle/ref_driver's grk_set_MCT: m00,m01,...:s0,s1,...
                    mv, sv = v.split(":")
                    p.set_mct([float(x) for x in mv.split(",")], [int(x) for x in sv.split(",")])
                elif a == "-d":
                    off = tuple(int(x) for x in v.split(","))
                elif a == "-p":
                    p.prog_order = PROGS[v[:4]]
                elif a in ("-R", "-ROI"):  # c=<comp>,U=<shift> (grk_compress.cpp:1470-1476)
                    kv = dict(x.split("=") for x in v.split(","))
                    p.roi_compno, p.roi_shift = int(kv["c"]), int(kv["U"])
                elif a == "-M":  # code-block mode switches (grk_compress.cpp:1132)
                    p.cblk_sty = int(v) & 0x7F
                elif a == "-A":
                    p.rate_control_algorithm = int(v)
                elif a == "-u":
                    p.tp_on = 1
                    p.tp_flag = ord(v[0])
                elif a in ("-r", "-q"):
                    vals = [float(x) for x in v.split(",")]
                    p.tcp_numlayers = len(vals)
                    for k, x in enumerate(vals):
                        if a == "-r":
                            p.tcp_rates[k] = 0.0 if x == 1 else x
                        else:
                            p.tcp_distoratio[k] = x
                    if a == "-r":
                        p.cp_disto_alloc = 1
                    else:
                        p.cp_fixed_quality = 1
                elif a == "-c":
                    sizes = [tuple(int(y) for y in t.strip("[]").split(",")) for t in v.replace("],[", "];[").split(";")]
                    p.csty |= CSTY_PRT
                    p.res_spec = len(sizes)
                    for k, (w, h) in enumerate(sizes):
                        p.prcw_init[k], p.prch_init[k] = w, h
                elif a == "-P":
                    n = 0
                    for ent in v.split("/"):
                        t, rest = ent[1:].split("=")
                        r0, c0, l1, r1, c1, pr = rest.split(",")
                        p.POC[n] = Poc(int(t), int(r0), int(c0), int(l1), int(r1), int(c1), PROGS[pr[:4]])
                        n += 1
                    p.numpocs = n
                elif a in ("-cinema2K", "-cinema4K", "-w", "-x"):
                    cinema = PROFILE_CINEMA_2K if a in ("-cinema2K", "-w") else PROFILE_CINEMA_4K
                    p.framerate = int(v)
                else:
                    raise ValueError("unsupported grk_compress option %s" % a)
            i += 1
        if cinema:  # checkCinema (grk_compress.cpp:537-561)
            p.rsiz = cinema
            p.max_comp_size = 520833 if p.framerate == 48 else 1041666
            p.max_cs_size = 651041 if p.framerate == 48 else 1302083
        return p, off


SAMPLE_I32, SAMPLE_U8, SAMPLE_I8, SAMPLE_U16, SAMPLE_I16 = 0, 1, 2, 3, 4
_NP_FMT = {np.dtype(np.int32): SAMPLE_I32, np.dtype(np.uint8): SAMPLE_U8, np.dtype(np.int8): SAMPLE_I8,
           np.dtype(np.uint16): SAMPLE_U16, np.dtype(np.int16): SAMPLE_I16}


class Planes(ctypes.Structure):
    """grkgpu_planes: the image planes of grkgpu_compress_ex."""
    _fields_ = [("planes", ctypes.c_void_p * MAXC), ("sample_fmt", ctypes.c_uint32), ("on_device", ctypes.c_int32),
                ("row0", ctypes.c_uint32), ("nrows", ctypes.c_uint32), ("col0", ctypes.c_uint32),
                ("ncols", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("h2d_ms", ctypes.c_float), ("dcshift_mct_ms", ctypes.c_float), ("dwt_ms", ctypes.c_float),
                ("t1_ms", ctypes.c_float), ("gather_ms", ctypes.c_float), ("d2h_ms", ctypes.c_float),
                ("host_t2_ms", ctypes.c_float), ("total_ms", ctypes.c_float), ("num_cblks", ctypes.c_uint64),
                ("cs_bytes", ctypes.c_uint64), ("mq_symbols", ctypes.c_uint64), ("rate_ms", ctypes.c_float),
                ("packet_ms", ctypes.c_float), ("rate_probes", ctypes.c_uint32), ("rate_probes_skipped", ctypes.c_uint32),
                ("rate_block_evals", ctypes.c_uint64), ("rate_precinct_sims", ctypes.c_uint64),
                ("rate_form_ms", ctypes.c_float), ("rate_sim_ms", ctypes.c_float), ("passrec_ms", ctypes.c_float),
                ("pad_", ctypes.c_uint32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class DwtOptions(ctypes.Structure):
    """grkgpu_dwt_options (include/grk_mi355x.h)."""
    _fields_ = [("fuse_level0", ctypes.c_int32), ("f01_rows", ctypes.c_int32), ("f01_min_samples", ctypes.c_uint64),
                ("f01_small_min_samples", ctypes.c_uint64), ("inv01", ctypes.c_int32), ("pair_group", ctypes.c_int32),
                ("inv01_min_samples", ctypes.c_uint64), ("f64_lift", ctypes.c_int32), ("t1_dec_sort", ctypes.c_int32),
                ("t1_dec_bpw", ctypes.c_int32), ("mid_th", ctypes.c_int32),
                ("t1_enc_bpw", ctypes.c_int32), ("t1_enc_sort", ctypes.c_int32), ("pair_kernel", ctypes.c_int32),
                ("pair_rows", ctypes.c_int32), ("pair_waves", ctypes.c_int32), ("pair_min_samples", ctypes.c_uint64)]


class DeviceSet(ctypes.Structure):
    """grkgpu_device_set (include/grk_mi355x.h): the device workers of a
    multi-device call (a device may repeat)."""
    _fields_ = [("n", ctypes.c_uint32), ("dev", ctypes.c_int32 * 64)]


class LaunchTime(ctypes.Structure):
    """grkgpu_launch_time (include/grk_mi355x.h)."""
    _fields_ = [("kernel", ctypes.c_char * 48), ("level0", ctypes.c_uint32), ("levels", ctypes.c_uint32),
                ("ms", ctypes.c_float), ("pad", ctypes.c_uint32), ("bytes", ctypes.c_uint64)]


_lib = None
_EXPORTS = None


def build():
    """Compile libgrk_mi355x.so for gfx950 (hipcc cross-compiles without a GPU) and the
    minpf plugin libgrok_plugin.so, in-tree."""
    import subprocess
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(_HERE, "csrc")], check=True)


def lib():
    global _lib
    if _lib is None:
        # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's); load
        # it first so the process has ONE HIP runtime shared by torch and us.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise GrkGpuError("libgrk_mi355x.so not built (run grokimagecompression_amd.build()); "
                              "there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        P, U32, I32, VP = ctypes.POINTER, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p
        L.grkgpu_version.restype = ctypes.c_char_p
        L.grkgpu_last_error.restype = ctypes.c_char_p
        L.grkgpu_create.argtypes = [ctypes.c_int, P(VP)]
        L.grkgpu_destroy.argtypes = [VP]
        L.grkgpu_set_stream.argtypes = [VP, VP]
        L.grkgpu_get_stats.argtypes = [VP, P(Stats)]
        L.grkgpu_set_launch_timing.argtypes = [VP, ctypes.c_int]
        L.grkgpu_get_dwt_options.argtypes = [P(DwtOptions)]
        L.grkgpu_get_dwt_options.restype = None
        L.grkgpu_set_dwt_options.argtypes = [P(DwtOptions)]
        L.grkgpu_get_launch_times.argtypes = [VP, P(LaunchTime), U32, P(U32)]
        L.grkgpu_device_set_for.argtypes = [ctypes.c_int, P(DeviceSet)]
        L.grkgpu_compress_multi.argtypes = [P(DeviceSet), P(ImageDesc), P(CParams), P(Planes), P(P(ctypes.c_uint8)),
                                            P(ctypes.c_size_t)]
        L.grkgpu_decompress_multi.argtypes = [P(DeviceSet), VP, ctypes.c_size_t, P(ImageDesc), P(VP)]
        L.grkgpu_patch_tlm.argtypes = [VP, ctypes.c_size_t]
        L.grkgpu_multi_release.argtypes = []
        L.grkgpu_multi_release.restype = None
        L.grkgpu_default_cparams.argtypes = [P(CParams)]
        L.grkgpu_set_mct.argtypes = [P(CParams), VP, VP, U32]
        L.grkgpu_compress.argtypes = [VP, P(ImageDesc), P(CParams), P(VP), ctypes.c_int, P(P(ctypes.c_uint8)),
                                      P(ctypes.c_size_t)]
        L.grkgpu_compress_view.argtypes = [VP, P(ImageDesc), P(CParams), P(VP), ctypes.c_int,
                                           P(P(ctypes.c_uint8)), P(ctypes.c_size_t)]
        L.grkgpu_compress_ex.argtypes = [VP, P(ImageDesc), P(CParams), P(Planes), U32, U32, U32, P(P(ctypes.c_uint8)),
                                         P(ctypes.c_size_t)]
        L.grkgpu_read_header.argtypes = [VP, ctypes.c_size_t, P(ImageDesc)]
        L.grkgpu_decompress.argtypes = [VP, VP, ctypes.c_size_t, P(ImageDesc), P(VP), ctypes.c_int]
        L.grkgpu_free.argtypes = [VP]
        L.grkgpu_take_output.argtypes = [VP, P(VP), P(ctypes.c_size_t)]
        L.grkgpu_give_output.argtypes = [VP, VP, ctypes.c_size_t]
        L.grkgpu_free_output.argtypes = [VP]
        L.grkgpu_free_output.restype = None
        L.grkgpu_num_tiles.argtypes = [P(ImageDesc), P(CParams), P(U32)]
        L.grkgpu_compress_tiles.argtypes = [VP, P(ImageDesc), P(CParams), P(VP), ctypes.c_int, U32, U32, U32,
                                            P(P(ctypes.c_uint8)), P(ctypes.c_size_t)]
        L.grkgpu_compress_tile_rows.argtypes = [VP, P(ImageDesc), P(CParams), P(VP), ctypes.c_int, U32, U32, U32, U32,
                                                U32, P(P(ctypes.c_uint8)), P(ctypes.c_size_t)]
        L.grkgpu_decompress_tiles.argtypes = [VP, VP, ctypes.c_size_t, U32, U32, P(VP), ctypes.c_int]
        L.grkgpu_walk_tiles.argtypes = [VP, ctypes.c_size_t, P(ctypes.c_uint8), U32, P(U32)]
        L.grkgpu_decompress_reduced.argtypes = [VP, VP, ctypes.c_size_t, U32, P(ImageDesc), P(VP), ctypes.c_int]
        L.grkgpu_decompress_window.argtypes = [VP, VP, ctypes.c_size_t, U32, U32, U32, U32, P(ImageDesc), P(VP),
                                               ctypes.c_int]
        L.grkgpu_decompress_ex.argtypes = [VP, VP, ctypes.c_size_t, P(DParams), P(ImageDesc), P(VP), ctypes.c_int]
        L.grkgpu_dcshift_mct_fwd.argtypes = [P(VP), U32, U32, U32, U32, P(I32), I32, I32, VP]
        L.grkgpu_mct_inv_dcshift.argtypes = [P(VP), U32, U32, U32, U32, P(U32), P(I32), I32, I32, VP]
        L.grkgpu_dwt_fwd.argtypes = [VP, VP, U32, U32, U32, U32, U32, I32, VP]
        L.grkgpu_dwt_inv.argtypes = [VP, VP, U32, U32, U32, U32, U32, I32, VP]
        L.grkgpu_dwt_scratch_bytes.restype = ctypes.c_size_t
        L.grkgpu_dwt_scratch_bytes.argtypes = [U32, U32, U32, U32, U32]
        L.grkgpu_t1_scratch_bytes.restype = ctypes.c_size_t
        L.grkgpu_t1_scratch_bytes_n.restype = ctypes.c_size_t
        L.grkgpu_t1_scratch_bytes_n.argtypes = [U32]
        L.grkgpu_t1_encode_blocks.argtypes = [VP, U32, VP, VP, VP, VP, ctypes.c_int, VP]
        L.grkgpu_t1_decode_blocks.argtypes = [VP, U32, VP, VP, VP, VP]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise GrkGpuError("grkgpu error %d: %s" % (rc, lib().grkgpu_last_error().decode()))


def _buf_ptr(buf):
    """(pointer, length, keepalive) of a codestream held in bytes / bytearray /
    numpy uint8 array, without copying."""
    if isinstance(buf, np.ndarray):
        assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        return ctypes.c_void_p(buf.ctypes.data), buf.size, buf
    if isinstance(buf, bytearray):
        arr = (ctypes.c_char * len(buf)).from_buffer(buf)
        return ctypes.cast(arr, ctypes.c_void_p), len(buf), arr
    if not isinstance(buf, bytes):
        buf = bytes(buf)
    cp = ctypes.c_char_p(buf)
    return ctypes.cast(cp, ctypes.c_void_p), len(buf), (cp, buf)


PART_TILES, PART_HEADER, PART_EOC, PART_ALL = 0, 1, 2, 3


def _fmt_fits(fmt, prec, sgnd):
    """Can samples of format fmt carry a (prec, sgnd) component at their own
    width (grkgpu_compress_ex's rule)?  Otherwise the caller widens to int32."""
    if fmt == SAMPLE_I32:
        return True
    bits = 8 if fmt in (SAMPLE_U8, SAMPLE_I8) else 16
    signed = fmt in (SAMPLE_I8, SAMPLE_I16)
    return bool(sgnd) == signed and prec <= bits


class _CtxView:
    """Owner of a numpy view of a context's pinned output buffer.  It takes
    the buffer out of the context (grkgpu_take_output: the Codec's next
    compress allocates its own, so later calls never overwrite or free these
    bytes) and gives it back when the last view or slice of it is gone
    (grkgpu_give_output; freed instead if the Codec was closed) -- numpy
    arrays made from __array_interface__ keep this object as their base, and
    every view of them keeps that base.  A caller that drops its view before
    the next compress (the bench) gets the same buffer back every time.  A
    caller that keeps views alive across compresses holds one pinned buffer
    (the codestream's size plus ~1/8) per live view; buffers given back while
    the context already has one are kept as spares (at most 4, the largest)
    and reused by later compresses instead of pinning new ones."""

    def __init__(self, codec, ptr, n):
        self.codec = codec
        self.buf, self.cap = ctypes.c_void_p(), ctypes.c_size_t()
        _check(lib().grkgpu_take_output(codec._ctx, ctypes.byref(self.buf), ctypes.byref(self.cap)))
        addr = ctypes.cast(ptr, ctypes.c_void_p).value
        self.__array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (addr, False), "version": 3}

    def __del__(self):
        try:
            if self.codec._ctx:
                lib().grkgpu_give_output(self.codec._ctx, self.buf, self.cap)
            else:
                lib().grkgpu_free_output(self.buf)
        except Exception:
            pass


def num_tiles(shape, prec, params, offset=(0, 0)):
    """Tile count of a (c,h,w) image under `params` (grkgpu_num_tiles)."""
    c, h, w = shape
    d = ImageDesc()
    d.x0, d.y0 = offset
    d.x1, d.y1 = offset[0] + w, offset[1] + h
    d.numcomps = c
    for k in range(c):
        d.prec[k] = prec
    n = ctypes.c_uint32()
    _check(lib().grkgpu_num_tiles(ctypes.byref(d), ctypes.byref(params), ctypes.byref(n)))
    return n.value


def read_header(buf):
    d = ImageDesc()
    ptr, n, keep = _buf_ptr(buf)
    _check(lib().grkgpu_read_header(ptr, n, ctypes.byref(d)))
    return d


def _torch():
    import torch
    return torch


def _check_out(out, shape, device):
    """Validate a caller-supplied output (shape, int32, contiguous, device)
    before raw pointers to it cross the C ABI."""
    if isinstance(out, np.ndarray):
        if out.shape != tuple(shape) or out.dtype != np.int32 or not out.flags.c_contiguous:
            raise GrkGpuError("out must be a C-contiguous int32 array of shape %s (got %s %s)"
                              % (tuple(shape), out.shape, out.dtype))
        return False
    torch = _torch()
    if not isinstance(out, torch.Tensor):
        raise GrkGpuError("out must be a numpy array or a torch tensor")
    if tuple(out.shape) != tuple(shape) or out.dtype != torch.int32 or not out.is_contiguous():
        raise GrkGpuError("out must be a contiguous int32 tensor of shape %s (got %s %s)"
                          % (tuple(shape), tuple(out.shape), out.dtype))
    if not out.is_cuda or out.device.index != device:
        raise GrkGpuError("out must live on cuda:%d (got %s)" % (device, out.device))
    return True


def _stream_handle(device):
    torch = _torch()
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Codec:
    """One HIP context (device, stream, device-memory arenas) per instance."""

    def __init__(self, device=0):
        self.device = device
        self._ctx = ctypes.c_void_p()
        _check(lib().grkgpu_create(device, ctypes.byref(self._ctx)))

    def close(self):
        if self._ctx:
            lib().grkgpu_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        s = Stats()
        _check(lib().grkgpu_get_stats(self._ctx, ctypes.byref(s)))
        return s.as_dict()

    def set_launch_timing(self, on=True):
        """Time every forward-DWT launch of later compress calls (HIP events)."""
        _check(lib().grkgpu_set_launch_timing(self._ctx, 1 if on else 0))

    def launch_times(self):
        """Forward-DWT launches of the last compress call: kernel, first level,
        level count, device ms, algorithmic bytes (grkgpu_get_launch_times)."""
        n = ctypes.c_uint32()
        _check(lib().grkgpu_get_launch_times(self._ctx, None, 0, ctypes.byref(n)))
        arr = (LaunchTime * max(1, n.value))()
        _check(lib().grkgpu_get_launch_times(self._ctx, arr, n.value, ctypes.byref(n)))
        return [{"kernel": t.kernel.decode(), "level0": t.level0, "levels": t.levels, "ms": t.ms, "bytes": t.bytes}
                for t in arr[:n.value]]

    def _image(self, img, prec, offset, sgnd):
        """Image descriptor + grkgpu_planes of a (c,h,w) numpy array or torch
        tensor of int32, uint16, int16, uint8 or int8 samples (host, pinned
        host, or on this codec's device)."""
        c, h, w = img.shape
        d = ImageDesc()
        d.x0, d.y0 = offset
        d.x1, d.y1 = offset[0] + w, offset[1] + h
        d.numcomps = c
        for k in range(c):
            d.prec[k] = prec
            d.sgnd[k] = 1 if sgnd else 0
        pl = Planes()
        if isinstance(img, np.ndarray):
            if img.dtype not in _NP_FMT or not _fmt_fits(_NP_FMT[img.dtype], prec, sgnd):
                img = img.astype(np.int32)
            img = np.ascontiguousarray(img)
            fmt = _NP_FMT[img.dtype]
            for k in range(c):
                pl.planes[k] = img[k].ctypes.data
            on_dev = False
        else:
            torch = _torch()
            tf = {torch.int32: SAMPLE_I32, torch.uint8: SAMPLE_U8, torch.int8: SAMPLE_I8, torch.int16: SAMPLE_I16}
            if hasattr(torch, "uint16"):
                tf[torch.uint16] = SAMPLE_U16
            if img.dtype not in tf or not img.is_contiguous():
                raise GrkGpuError("image tensor must be contiguous int32 / uint16 / int16 / uint8 / int8")
            if not _fmt_fits(tf[img.dtype], prec, sgnd):
                img = img.to(torch.int32)  # e.g. 12-bit unsigned samples held in int16
            fmt = tf[img.dtype]
            on_dev = img.is_cuda
            if on_dev:
                if img.device.index != self.device:
                    raise GrkGpuError("image tensor on %s, codec on cuda:%d" % (img.device, self.device))
                lib().grkgpu_set_stream(self._ctx, _stream_handle(img.device))
            else:
                # host tensor (pinned or not): the library copies it H2D on the
                # caller's current stream
                lib().grkgpu_set_stream(self._ctx, _stream_handle(torch.device("cuda", self.device)))
            for k in range(c):
                pl.planes[k] = img[k].data_ptr()
        pl.sample_fmt = fmt
        pl.on_device = 1 if on_dev else 0
        return d, pl, img

    def compress(self, img, prec, params=None, offset=(0, 0), sgnd=False, view=False):
        """img: (c,h,w) numpy array or torch tensor (host, pinned host or
        cuda:<device>) of int32 samples, or of the 8 / 16-bit samples of the
        image file (uint8 / int8 / uint16 / int16: widened on the GPU, so a host
        frame crosses PCIe at its own width).  Returns the .j2k codestream as
        bytes, or (view=True) as a zero-copy numpy uint8 view of the context's
        pinned output buffer, valid for as long as the view lives (_CtxView)."""
        return self.compress_tiles(img, prec, params or CParams.make(), 0, 0xFFFFFFFF, PART_ALL, offset, sgnd,
                                   view=view)

    def compress_subsampled(self, planes, prec, size, subsampling, params=None, offset=(0, 0), sgnd=False):
        """Subsampled components (SIZ XRsiz / YRsiz): planes[k] is component
        k's (h_k, w_k) array on its grid, component k subsampled by
        subsampling[k] = (dx, dy) of an image size = (w, h) at `offset` on the
        reference grid (w_k = ceil((x0 + w) / dx) - ceil(x0 / dx)); host numpy
        planes, int32 or their 8 / 16-bit samples.  MCT is disabled when the
        first three components differ in subsampling (j2k.cpp:1963-1971)."""
        c = len(planes)
        if len(subsampling) != c:
            raise GrkGpuError("one (dx, dy) per component")
        d = ImageDesc()
        d.x0, d.y0 = offset
        d.x1, d.y1 = offset[0] + size[0], offset[1] + size[1]
        d.numcomps = c
        pl = Planes()
        keep = []
        fmts = set()
        for k, (a, (dx, dy)) in enumerate(zip(planes, subsampling)):
            cw = -(-d.x1 // dx) - (-(-d.x0 // dx))
            ch = -(-d.y1 // dy) - (-(-d.y0 // dy))
            a = np.asarray(a)
            if a.shape != (ch, cw):
                raise GrkGpuError("component %d: plane %s, its grid needs %s" % (k, a.shape, (ch, cw)))
            if a.dtype not in _NP_FMT or not _fmt_fits(_NP_FMT[a.dtype], prec, sgnd):
                a = a.astype(np.int32)
            a = np.ascontiguousarray(a)
            keep.append(a)
            fmts.add(_NP_FMT[a.dtype])
            d.prec[k], d.sgnd[k], d.dx[k], d.dy[k] = prec, 1 if sgnd else 0, dx, dy
            pl.planes[k] = a.ctypes.data
        if len(fmts) != 1:
            keep = [a.astype(np.int32) for a in keep]
            for k, a in enumerate(keep):
                pl.planes[k] = a.ctypes.data
            fmts = {SAMPLE_I32}
        pl.sample_fmt = fmts.pop()
        pl.on_device = 0
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        _check(lib().grkgpu_compress_ex(self._ctx, ctypes.byref(d), ctypes.byref(params or CParams.make()),
                                        ctypes.byref(pl), 0, 0xFFFFFFFF, PART_ALL, ctypes.byref(out), ctypes.byref(n)))
        return ctypes.string_at(out, n.value)

    def compress_tiles(self, img, prec, params, tile_begin, tile_end, parts=PART_TILES, offset=(0, 0), sgnd=False,
                       row0=None, height=None, view=False):
        """Encode tiles [tile_begin, tile_end) of img; returns their tile-parts
        (plus the main header / EOC when `parts` asks for them) as bytes, or
        (view=True) as a numpy uint8 view of the context's pinned output
        buffer (no copy), valid for as long as the view lives (_CtxView).
        row0 / height: img holds only image rows [row0, row0 + img rows) of an
        image `height` rows tall (a tile-row shard)."""
        d, pl, keep = self._image(img, prec, offset, sgnd)
        if row0 is not None:
            if height is None:
                raise GrkGpuError("height (the full image height) is required with row0")
            d.y1 = offset[1] + height
            pl.row0, pl.nrows = row0, img.shape[1]
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        _check(lib().grkgpu_compress_ex(self._ctx, ctypes.byref(d), ctypes.byref(params), ctypes.byref(pl), tile_begin,
                                        tile_end, parts, ctypes.byref(out), ctypes.byref(n)))
        if view:
            return np.asarray(_CtxView(self, out, n.value)) if n.value else np.empty(0, np.uint8)
        return ctypes.string_at(out, n.value)

    def decompress_tiles(self, buf, tile_begin, tile_end, out):
        """Decode tiles [tile_begin, tile_end) of a codestream into `out`
        ((c,h,w) int32 numpy array or cuda tensor); other tiles untouched."""
        d = read_header(buf)
        c = d.numcomps
        on_dev = _check_out(out, (c, d.y1 - d.y0, d.x1 - d.x0), self.device)
        if on_dev:
            lib().grkgpu_set_stream(self._ctx, _stream_handle(out.device))
            ptrs = (ctypes.c_void_p * c)(*[out[k].data_ptr() for k in range(c)])
        else:
            ptrs = (ctypes.c_void_p * c)(*[out[k].ctypes.data for k in range(c)])
        bp, bn, keep = _buf_ptr(buf)
        _check(lib().grkgpu_decompress_tiles(self._ctx, bp, bn, tile_begin, tile_end, ptrs, 1 if on_dev else 0))
        return out

    def decompress(self, buf, device_out=False, out=None, reduce=0, window=None, layers=0):
        """Decode a .j2k codestream -> (c,h,w) int32 (numpy, or torch.cuda when
        device_out / out is a cuda tensor).  reduce > 0: the image at
        resolution numres-1-reduce (grk_decompress -r), ceil(size / 2^reduce)
        samples a side (a window: ceil(x1 / 2^reduce) - ceil(x0 / 2^reduce)).  window = (x0, y0, x1, y1) in image coordinates:
        only that region (grk_set_decode_area), clipped to the image.
        layers > 0: only the first `layers` quality layers (grk_decompress -l)."""
        d = read_header(buf)
        if window is not None:  # the window (reference grid) clipped to the image
            wx0, wy0, wx1, wy1 = window
            d.x0, d.y0, d.x1, d.y1 = max(d.x0, wx0), max(d.y0, wy0), min(d.x1, wx1), min(d.y1, wy1)
            if d.x1 <= d.x0 or d.y1 <= d.y0:
                raise GrkGpuError("decode window outside the image")
        # planes at the decoded resolution: a window's extent
        # ceil(x1 / 2^r) - ceil(x0 / 2^r) (update_image_dimensions); the whole
        # image's ceil(size / 2^r) (grk_image_comp_header_update), the
        # decoded samples placed from ceil(x0 / 2^r) and the rest zero
        cd = lambda v, s: -(-v // s)  # noqa: E731
        R = 1 << reduce

        def extent(a0, a1, s):
            if window is not None:
                return cd(cd(a1, s), R) - cd(cd(a0, s), R)
            return cd(cd(a1, s) - cd(a0, s), R)
        c = d.numcomps
        h, w = extent(d.y0, d.y1, 1), extent(d.x0, d.x1, 1)
        if any(d.dx[k] != 1 or d.dy[k] != 1 for k in range(c)):
            # subsampled components: a list of host planes, each on its grid
            if out is not None or device_out:
                raise GrkGpuError("subsampled components decode to host planes only")
            outs = [np.empty((extent(d.y0, d.y1, d.dy[k]), extent(d.x0, d.x1, d.dx[k])), dtype=np.int32)
                    for k in range(c)]
            ptrs = (ctypes.c_void_p * c)(*[a.ctypes.data for a in outs])
            bp, bn, keep = _buf_ptr(buf)
            dp = DParams(cp_reduce=reduce, cp_layer=layers)
            if window is not None:
                dp.DA_x0, dp.DA_y0, dp.DA_x1, dp.DA_y1 = [int(v) for v in window]
            _check(lib().grkgpu_decompress_ex(self._ctx, bp, bn, ctypes.byref(dp), None, ptrs, 0))
            return outs
        if out is not None:
            on_dev = _check_out(out, (c, h, w), self.device)
        else:
            on_dev = bool(device_out)
        if on_dev:
            torch = _torch()
            if out is None:
                out = torch.empty((c, h, w), dtype=torch.int32, device="cuda:%d" % self.device)
            lib().grkgpu_set_stream(self._ctx, _stream_handle(out.device))
            ptrs = (ctypes.c_void_p * c)(*[out[k].data_ptr() for k in range(c)])
        else:
            if out is None:
                out = np.empty((c, h, w), dtype=np.int32)
            ptrs = (ctypes.c_void_p * c)(*[out[k].ctypes.data for k in range(c)])
        bp, bn, keep = _buf_ptr(buf)
        if layers < 0:
            raise GrkGpuError("layers must be >= 0")
        if window is not None or reduce or layers:
            dp = DParams(cp_reduce=reduce, cp_layer=layers)
            if window is not None:
                dp.DA_x0, dp.DA_y0, dp.DA_x1, dp.DA_y1 = [int(v) for v in window]
            _check(lib().grkgpu_decompress_ex(self._ctx, bp, bn, ctypes.byref(dp), None, ptrs, 1 if on_dev else 0))
        else:
            _check(lib().grkgpu_decompress(self._ctx, bp, bn, None, ptrs, 1 if on_dev else 0))
        return out


def device_set(device=-1):
    """The device workers grkgpu_device_set_for picks: [device] for device >= 0;
    for -1 ("all devices", grk_cparameters.deviceId) the GRKGPU_DEVICES list
    ("0,1" / "0,0" / "all"), else every visible device."""
    ds = DeviceSet()
    _check(lib().grkgpu_device_set_for(device, ctypes.byref(ds)))
    return list(ds.dev[:ds.n])


def _devset(devices):
    ds = DeviceSet()
    if devices is None:
        _check(lib().grkgpu_device_set_for(-1, ctypes.byref(ds)))
        return ds
    devices = list(devices)
    if not 0 < len(devices) <= 64:
        raise GrkGpuError("1 .. 64 device workers")
    ds.n = len(devices)
    for k, v in enumerate(devices):
        ds.dev[k] = v
    return ds


def compress_multi(img, prec, params=None, devices=None, offset=(0, 0), sgnd=False):
    """One encode over several device workers (grkgpu_compress_multi: the
    tiles sharded in contiguous ranges, each worker uploading only its tiles'
    rows; the pieces concatenated in tile order, TLM patched).  img: (c,h,w)
    host numpy array (int32 or the file's 8 / 16-bit samples).  devices: the
    workers' devices (a device may repeat), default device_set(-1).  Returns
    the codestream bytes -- the same bytes as Codec.compress."""
    c, h, w = img.shape
    d = ImageDesc()
    d.x0, d.y0 = offset
    d.x1, d.y1 = offset[0] + w, offset[1] + h
    d.numcomps = c
    for k in range(c):
        d.prec[k] = prec
        d.sgnd[k] = 1 if sgnd else 0
    if img.dtype not in _NP_FMT or not _fmt_fits(_NP_FMT[img.dtype], prec, sgnd):
        img = img.astype(np.int32)
    img = np.ascontiguousarray(img)
    pl = Planes()
    for k in range(c):
        pl.planes[k] = img[k].ctypes.data
    pl.sample_fmt = _NP_FMT[img.dtype]
    pl.on_device = 0
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    ds = _devset(devices)
    _check(lib().grkgpu_compress_multi(ctypes.byref(ds), ctypes.byref(d), ctypes.byref(params or CParams.make()),
                                       ctypes.byref(pl), ctypes.byref(out), ctypes.byref(n)))
    try:
        return ctypes.string_at(out, n.value)
    finally:
        lib().grkgpu_free(out)


def decompress_multi(buf, devices=None, out=None):
    """Whole-image decode over several device workers (grkgpu_decompress_multi:
    each decodes its tile range) into a (c,h,w) int32 host array."""
    d = read_header(buf)
    c = d.numcomps
    shape = (c, d.y1 - d.y0, d.x1 - d.x0)
    if out is None:
        out = np.empty(shape, dtype=np.int32)
    elif _check_out(out, shape, 0):
        raise GrkGpuError("decompress_multi writes host planes")
    ptrs = (ctypes.c_void_p * c)(*[out[k].ctypes.data for k in range(c)])
    bp, bn, keep = _buf_ptr(buf)
    ds = _devset(devices)
    _check(lib().grkgpu_decompress_multi(ctypes.byref(ds), bp, bn, None, ptrs))
    return out


class dwt_options:
    """Context manager over the process-wide DWT plan options
    (grkgpu_set_dwt_options): e.g. ``with dwt_options(fuse_level0=0): ...``
    runs the block with the separate DC shift / MCT pass; the previous options
    come back on exit.  The defaults are the plans measured fastest."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.old = DwtOptions()
        lib().grkgpu_get_dwt_options(ctypes.byref(self.old))
        new = DwtOptions()
        ctypes.pointer(new)[0] = self.old
        for k, v in self.kw.items():
            setattr(new, k, v)
        _check(lib().grkgpu_set_dwt_options(ctypes.byref(new)))
        return self

    def __exit__(self, *exc):
        _check(lib().grkgpu_set_dwt_options(ctypes.byref(self.old)))
        return False


def walk_tiles(cs):
    """The tile-part walk of a decode of codestream bytes `cs`, host only
    (grkgpu_walk_tiles): the list of tiles a decode produces; raises
    GrkGpuError where the decode fails in the walk."""
    n = ctypes.c_uint32()
    buf = ctypes.create_string_buffer(bytes(cs), len(cs))
    _check(lib().grkgpu_walk_tiles(buf, len(cs), None, 0, ctypes.byref(n)))
    dec = (ctypes.c_uint8 * max(1, n.value))()
    _check(lib().grkgpu_walk_tiles(buf, len(cs), dec, n.value, ctypes.byref(n)))
    return [t for t in range(n.value) if dec[t]]


# ---- stage entry points on torch device tensors (per-kernel parity tests) ----

def dwt_fwd(t, x0, y0, numres, irreversible):
    """In-place forward DWT of a (h,w) int32 cuda tensor (Mallat layout)."""
    torch = _torch()
    h, w = t.shape
    scratch = torch.empty(lib().grkgpu_dwt_scratch_bytes(x0, y0, x0 + w, y0 + h, numres) // 4 + 64, dtype=torch.int32, device=t.device)
    _check(lib().grkgpu_dwt_fwd(t.data_ptr(), scratch.data_ptr(), x0, y0, x0 + w, y0 + h, numres,
                                1 if irreversible else 0, _stream_handle(t.device)))
    return t


def dwt_inv(t, x0, y0, numres, irreversible):
    torch = _torch()
    h, w = t.shape
    scratch = torch.empty(lib().grkgpu_dwt_scratch_bytes(x0, y0, x0 + w, y0 + h, numres) // 4 + 64, dtype=torch.int32, device=t.device)
    _check(lib().grkgpu_dwt_inv(t.data_ptr(), scratch.data_ptr(), x0, y0, x0 + w, y0 + h, numres,
                                1 if irreversible else 0, _stream_handle(t.device)))
    return t


def dcshift_mct_fwd(planes, shifts, mct, irreversible):
    """planes: (c,h,w) int32 cuda tensor, modified in place."""
    c, h, w = planes.shape
    ptrs = (ctypes.c_void_p * c)(*[planes[k].data_ptr() for k in range(c)])
    sh = (ctypes.c_int32 * c)(*shifts)
    _check(lib().grkgpu_dcshift_mct_fwd(ptrs, c, w, h, w, sh, mct, 1 if irreversible else 0,
                                        _stream_handle(planes.device)))
    return planes


def mct_inv_dcshift(planes, prec, sgnd, mct, irreversible):
    c, h, w = planes.shape
    ptrs = (ctypes.c_void_p * c)(*[planes[k].data_ptr() for k in range(c)])
    pr = (ctypes.c_uint32 * c)(*([prec] * c))
    sg = (ctypes.c_int32 * c)(*([1 if sgnd else 0] * c))
    _check(lib().grkgpu_mct_inv_dcshift(ptrs, c, w, h, w, pr, sg, mct, 1 if irreversible else 0,
                                        _stream_handle(planes.device)))
    return planes
