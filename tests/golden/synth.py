"""Deterministic, integer-only synthetic image generator.

Test/bench infrastructure (not product code).  Every value is produced with
exact integer arithmetic (splitmix64 noise + triangle-wave "smooth" field), so
the same (shape, bits, seed, kind) gives bit-identical images on any host/CPU
(no libm, no SIMD-dependent float paths).  The golden codestreams under
tests/golden/ were produced by feeding these images to the reference
grk_compress (see oracle/make_golden.py), so the generator IS part of the
fixture definition: tests check sha256(image) against the recorded value.

Kinds (BASELINE.md "Inputs"):
  smooth   - smooth field + ~2% noise (primary)
  uniform  - uniform full-range noise (worst case for MQ)
  const    - constant mid-grey (numbps == 0 code-blocks)
"""
import hashlib
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    """Vectorised splitmix64 finaliser over a uint64 array (wrapping)."""
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def _noise(h, w, seed, comp, rows=None):
    r0, r1 = (0, h) if rows is None else rows
    idx = (np.arange(r0 * w, r1 * w, dtype=np.uint64)
           + np.uint64((seed * 1000003 + comp * 7919) << 32))
    with np.errstate(over="ignore"):
        return splitmix64(idx).reshape(r1 - r0, w)


def synth_plane(h, w, bits, seed, comp=0, kind="smooth", signed=False, rows=None):
    """One component plane as int32 (unsigned range [0, 2^bits-1], or signed
    range [-2^(bits-1), 2^(bits-1)-1] when signed=True)."""
    maxv = (1 << bits) - 1
    r0, r1 = (0, h) if rows is None else rows
    if kind == "const":
        v = np.full((r1 - r0, w), maxv // 2, dtype=np.int64)
    elif kind == "uniform":
        v = (_noise(h, w, seed, comp, (r0, r1)) % np.uint64(maxv + 1)).astype(np.int64)
    elif kind == "smooth":
        y = np.arange(r0, r1, dtype=np.int64)[:, None]
        x = np.arange(w, dtype=np.int64)[None, :]
        p1 = 97 + 13 * comp
        p2 = 71 + 7 * comp
        t1 = np.abs((3 * x + 17 * comp) % (2 * p1) - p1)          # 0..p1
        t2 = np.abs((2 * y + 29 * comp) % (2 * p2) - p2)          # 0..p2
        # base in [maxv/8, 7*maxv/8] plus gentle ramps
        base = (maxv * (t1 * p2 + t2 * p1)) // (2 * p1 * p2)      # 0..maxv
        base = base * 5 // 8 + maxv // 8
        base = base + (maxv * x) // (5 * max(w, 1)) - (maxv * y) // (10 * max(h, 1))
        amp = max(1, (maxv * 2) // 100)
        nz = (_noise(h, w, seed, comp, (r0, r1)) % np.uint64(2 * amp + 1)).astype(np.int64) - amp
        v = np.clip(base + nz, 0, maxv)
    else:
        raise ValueError(kind)
    if signed:
        v = v - (1 << (bits - 1))
    return v.astype(np.int32)


def synth_image(h, w, ncomp, bits, seed, kind="smooth", signed=False):
    """(ncomp, h, w) int32 planar image."""
    return np.stack([synth_plane(h, w, bits, seed, c, kind, signed) for c in range(ncomp)])


def image_sha256(img):
    return hashlib.sha256(np.ascontiguousarray(img, dtype=np.int32).tobytes()).hexdigest()


def write_pnm(path, img, bits):
    """img: (ncomp, h, w), ncomp in {1,3}, unsigned."""
    c, h, w = img.shape
    magic = b"P6" if c == 3 else b"P5"
    a = np.transpose(img, (1, 2, 0))
    with open(path, "wb") as f:
        f.write(magic + b"\n%d %d\n%d\n" % (w, h, (1 << bits) - 1))
        if bits <= 8:
            f.write(a.astype(np.uint8).tobytes())
        else:
            f.write(a.astype(">u2").tobytes())


def write_raw(path, img, bits):
    """Planar big-endian raw (grk_compress -F ...); signed allowed."""
    c, h, w = img.shape
    with open(path, "wb") as f:
        for k in range(c):
            if bits <= 8:
                f.write(img[k].astype(np.int8 if img.min() < 0 else np.uint8).tobytes())
            else:
                f.write(img[k].astype(">i2" if img.min() < 0 else ">u2").tobytes())
