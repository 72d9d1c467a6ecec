"""Multi-device calls behind the C ABI (grkgpu_compress_multi /
grkgpu_decompress_multi; grk_encode with grk_cparameters.deviceId = -1 and
grk_decode with GRKGPU_DEVICES): one call shards the tiles over several device
workers -- a host thread and a context each -- and concatenates the tile-parts
in tile order (the reference's tile loop
j2k.cpp:2088-2111, "-1 = all devices" grk_compress.cpp:423-426).

The box has one GPU, so the workers are listed explicitly on device 0
(devices=[0, 0] / GRKGPU_DEVICES=0,0): the sharding, the row windows each
worker uploads, the concatenation and the per-range decodes are the same as
on eight devices.  Bar: the reference's bytes and decoded samples exactly.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

import synth
from conftest import GOLD, ROOT, load_manifest

pytestmark = pytest.mark.gpu
MAN = load_manifest()
LARGE = load_manifest(large=True)
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver_mi355x")
TILED = sorted(n for n in MAN if "-t" in MAN[n]["args"])


def _img(m):
    h, w, c, bits = m["shape"]
    img = synth.synth_image(h, w, c, bits, m["seed"], m["kind"])
    assert synth.image_sha256(img) == m["image_sha256"]
    return img, bits


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], [0] * 5])
@pytest.mark.parametrize("name", TILED + ["rgb12_I", "rgb12_cinema4k"])
def test_multi_encode_decode_match_reference(name, devices):
    """Every tiled golden (and two single-tile ones: one worker does it all)
    through 2, 3 and 5 workers: the reference's codestream byte for byte, and
    the tile-range decodes assemble the reference's decoded image."""
    import grokimagecompression_amd as grk
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    b = grk.compress_multi(img, bits, p, devices=devices, offset=off)
    assert b == gold
    d = grk.decompress_multi(gold, devices=devices)
    assert np.array_equal(d, np.load(f"{GOLD}/{name}.dec.npy"))


def test_multi_planes_as_file_samples():
    """16-bit file samples (grkgpu_planes sample_fmt U16) through the
    workers' row windows: the same bytes as from int32 planes."""
    import grokimagecompression_amd as grk
    m = MAN["g8_tiles64"]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    assert grk.compress_multi(img.astype(np.uint8), bits, p, devices=[0, 0], offset=off) == \
        open(f"{GOLD}/g8_tiles64.j2k", "rb").read()


def test_multi_c4_full_size():
    """C4 (16384^2 16-bit, 256 tiles of 1024^2, 7 resolutions) through two
    workers: the reference's codestream hash; the two-range decode is the
    source image (lossless)."""
    import grokimagecompression_amd as grk
    m = LARGE["C4_16k_gray16_tiled"]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    b = grk.compress_multi(img.astype(np.uint16), bits, p, devices=[0, 0], offset=off)
    assert hashlib.sha256(b).hexdigest() == m["j2k_sha256"]
    d = grk.decompress_multi(b, devices=[0, 0])
    assert np.array_equal(d, img)


def _need_driver():
    if not os.path.exists(DRIVER):
        pytest.skip("oracle/_ref/ref_driver_mi355x not built (needs /root/reference at build time)")


def _drive(args, env_devices, tmp_path, img=None, shape=None):
    env = dict(os.environ, GRKGPU_DEVICES=env_devices)
    return subprocess.run([DRIVER] + args, capture_output=True, text=True, timeout=600, env=env)


@pytest.mark.parametrize("name", TILED)
def test_grk_api_all_devices(name, tmp_path):
    """grk_compress's library calls with -G -1 (grk_cparameters.deviceId =
    -1) and grk_decompress's with GRKGPU_DEVICES naming the workers: the
    reference's fixture driver relinked against our libgrok.so gives the
    reference's bytes and samples."""
    _need_driver()
    m = MAN[name]
    h, w, c, bits = m["shape"]
    img, _ = _img(m)
    src, out, dec = tmp_path / "in.i32", tmp_path / "out.j2k", tmp_path / "out.i32"
    np.ascontiguousarray(img, dtype="<i4").tofile(src)
    r = _drive(["enc", str(src), str(out), str(w), str(h), str(c), str(bits), "0"] + m["args"] + ["-G", "-1"],
               "0,0", tmp_path)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == open(f"{GOLD}/{name}.j2k", "rb").read()
    r = _drive(["dec", str(out), str(dec)], "0,0,0", tmp_path)
    assert r.returncode == 0, r.stderr
    x0, y0, x1, y1, nc, prec, sgnd, cw, ch = map(int, r.stdout.splitlines()[0].split())
    assert np.array_equal(np.fromfile(dec, dtype="<i4").reshape(nc, ch, cw), np.load(f"{GOLD}/{name}.dec.npy"))


def test_grk_api_all_devices_c4(tmp_path):
    """The verdict's bar: grk_encode of C4 with deviceId = -1 over two
    workers gives the reference hash, and grk_decode of it the source image."""
    _need_driver()
    m = LARGE["C4_16k_gray16_tiled"]
    h, w, c, bits = m["shape"]
    img, _ = _img(m)
    src, out, dec = tmp_path / "in.i32", tmp_path / "out.j2k", tmp_path / "out.i32"
    np.ascontiguousarray(img, dtype="<i4").tofile(src)
    r = _drive(["enc", str(src), str(out), str(w), str(h), str(c), str(bits), "0"] + m["args"] + ["-G", "-1"],
               "0,0", tmp_path)
    assert r.returncode == 0, r.stderr
    assert hashlib.sha256(out.read_bytes()).hexdigest() == m["j2k_sha256"]
    os.unlink(src)
    r = _drive(["dec", str(out), str(dec)], "0,0", tmp_path)
    assert r.returncode == 0, r.stderr
    assert synth.image_sha256(np.fromfile(dec, dtype="<i4").reshape(c, h, w)) == m["image_sha256"]
