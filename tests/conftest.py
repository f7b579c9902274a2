import glob
import json
import os
import sys

import pytest

try:  # one HIP runtime per process: torch's bundled runtime must be loaded before the library
    import torch  # noqa: F401  (libngram_search.so then binds to it by SONAME)
except ImportError:  # pragma: no cover
    torch = None

# a box here has one GPU: the multi-replica tests place several replicas on device 0, and the library
# splits a batch only over replicas on distinct devices unless told to split over every replica
os.environ.setdefault("NGS_SPLIT_SAME_DEVICE", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


def load_fixtures():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.json"))):
        with open(p) as f:
            out.append(json.load(f))
    return out


def fixture_words(fx):
    return [None if w is None else w.encode("latin-1") for w in fx["words"]]


def fixture_weights(fx):
    import struct
    if fx["weights"] is None:
        return None
    return [struct.unpack("<f", struct.pack("<I", b))[0] for b in fx["weights"]]


@pytest.fixture(scope="session")
def fixtures():
    return load_fixtures()
