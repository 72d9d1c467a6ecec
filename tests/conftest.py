import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, GOLD, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


# grk_compress options the round-1 C oracle restates (default coding style:
# one layer, LRCP, maximal precincts); the round-2 fixtures (layers / rate
# control, precincts, progressions, POC, SOP / EPH, tile-parts, cinema) are
# pinned by the reference itself (tests/test_ref_pinning.py) and checked on
# the GPU path against the reference's bytes.
ORACLE_OPTS = {"-I", "-n", "-b", "-t", "-T", "-Y", "-d"}


def oracle_supported(args):
    return all(a in ORACLE_OPTS for a in args if a.startswith("-"))


def load_manifest(large=False):
    return json.load(open(os.path.join(GOLD, "manifest_large.json" if large else "manifest.json")))


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def codec():
    import grokimagecompression_amd as grk
    c = grk.Codec(0)
    yield c
    c.close()
