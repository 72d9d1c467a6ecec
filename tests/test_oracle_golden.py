"""The CPU oracle is pinned against reference-generated codestreams.

tests/golden/*.j2k were written by the reference grk_compress (Grok v5.1.0)
from tests/golden/synth.py images (oracle/make_golden.py); *.dec.npy are the
reference grk_decompress outputs.  The oracle must reproduce both exactly.
"""
import hashlib

import numpy as np
import pytest

import synth
from conftest import GOLD, load_manifest

MAN = load_manifest()


@pytest.mark.parametrize("name", sorted(MAN))
def test_oracle_encode_matches_reference(oracle, name):
    m = MAN[name]
    h, w, c, bits = m["shape"]
    img = synth.synth_image(h, w, c, bits, m["seed"], m["kind"])
    assert synth.image_sha256(img) == m["image_sha256"], "generator drift"
    p = oracle.params_from_args(m["args"], nthreads=4)
    b = oracle.encode(img, bits, p, oracle.image_offset_from_args(m["args"]))
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    assert hashlib.sha256(gold).hexdigest() == m["j2k_sha256"]
    assert b == gold


@pytest.mark.parametrize("name", sorted(MAN))
def test_oracle_decode_matches_reference(oracle, name):
    gold = open(f"{GOLD}/{name}.j2k", "rb").read()
    ref = np.load(f"{GOLD}/{name}.dec.npy")
    d = oracle.decode(gold, nthreads=4)
    assert d.shape == ref.shape
    assert np.array_equal(d, ref)


def test_oracle_lossless_roundtrip_random(oracle):
    rng = np.random.default_rng(7)
    for (h, w, c, bits) in [(33, 47, 1, 8), (19, 70, 3, 12), (64, 64, 3, 16)]:
        img = rng.integers(0, 1 << bits, size=(c, h, w)).astype(np.int32)
        b = oracle.encode(img, bits, oracle.params(numres=4))
        assert np.array_equal(oracle.decode(b), img)
