"""ngsServe: single score()/search() calls answered by the persistent low-latency server kernel.

The server must give the regular path's answers bit for bit (and so the oracle's): every golden
fixture with its validChar phases, a seeded C1-shaped corpus (1k rows, BASELINE configs[0]) with
long, short, lower-case, wildcard and empty queries over several thresholds and limits, and
calls that fall back to the regular path (limit 0 or above 128). The kernel leaves after its idle
time and is relaunched on the next call; dispose stops it.
"""
import time

import pytest

from conftest import fixture_weights, fixture_words, load_fixtures
from oracle_py import OracleIndex
from test_gpu_parity import assert_exact

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu


def test_serve_matches_regular_path_c1_shape():
    words, _, rng = ssl.synth.gen_corpus(1000, seed=42)
    qs = ssl.synth.gen_queries(words, 1, 200, rng)
    qs += [w for w in words[:10]] + [w.lower() for w in words[10:14]] + [w[:5] for w in words[14:20]]
    qs += [w[:3] for w in words[20:24]] + [b"", b"*", b"  ", b"###", b"AB", b"z"]
    gi = ssl.StringIndex(words, 1, None)
    oi = OracleIndex(words, 1, None)
    cases = [(0.0, 100), (0.3, 100), (0.5, 10), (0.3, 128), (0.3, 129), (0.3, 0)]
    want = {(q, t, l): gi.score(q, t, l) for q in qs for t, l in cases}
    gi.serve(True)
    for q in qs:
        for t, l in cases:
            got = gi.score(q, t, l)
            assert got == want[(q, t, l)], f"served q={q!r} thr={t} limit={l}"
            assert_exact(got, oi.score(q, t, l), f"served vs oracle q={q!r} thr={t} limit={l}")
            assert gi.search(q, t, l) == [k for k, _ in got]
    # idle past the server's 200 ms: it leaves, the next call relaunches it
    time.sleep(0.5)
    for q in qs[:20]:
        assert gi.score(q, 0.3, 100) == want[(q, 0.3, 100)]
    gi.serve(False)
    assert gi.score(qs[0], 0.3, 100) == want[(qs[0], 0.3, 100)]
    gi.serve(True)
    gi.dispose()  # stops the server first


@pytest.mark.parametrize("fx", load_fixtures(), ids=lambda f: f["name"])
def test_serve_fixtures(fx):
    words, weights = fixture_words(fx), fixture_weights(fx)
    plain = ssl.StringIndex(words, fx["rowSize"], weights)
    served = ssl.StringIndex(words, fx["rowSize"], weights)
    served.serve(True)
    for ph in fx["phases"]:
        if ph["validChar"] is not None:
            plain.set_valid_char(ph["validChar"].encode("latin-1"))
            served.set_valid_char(ph["validChar"].encode("latin-1"))
        for c in ph["cases"]:
            q = c["q"].encode("latin-1")
            import struct
            thr = struct.unpack("<f", struct.pack("<I", c["thr"]))[0]
            assert served.score(q, thr, c["limit"]) == plain.score(q, thr, c["limit"]), f"{fx['name']} q={q!r}"
    plain.dispose()
    served.dispose()
