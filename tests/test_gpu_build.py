"""GPU index build against the host build of the same arrays (ngs_index.cpp):
* ngs_build.hip (gram CSR + skip table from the terms in HBM) vs NGS_HOST_GRAMS=1;
* ngs_intern.hip (interning, term ids, key ranks, term -> key CSR, wildcard weights) vs
  NGS_HOST_INTERN=1, on narrow and wide libraries with aliases, NULL words, blank keys, repeated
  (term, key) pairs with different weights (last write wins, nGramSearch.hpp:146-147), zero and
  negative weights, escaped and lower-case characters.

Both must be bit-identical (ngsIndexDigest: FNV-1a of every array as the kernels read it),
answer getSize / getLibSize alike, and search alike; covers dense lists (more than 256 skip
buckets), repeated grams inside a term, short / long term mixes and an empty long library.
"""
import ctypes as C
import os
import random

import pytest

import stringsearchlib_amd as ssl
from stringsearchlib_amd import _native

pytestmark = pytest.mark.gpu


def _digest(idx):
    out = (C.c_uint64 * 17)()
    assert _native.lib().ngsIndexDigest(idx.handle, out, 17) == 17
    return list(out)


def _build(words, rs=1, wts=None, host=False, env="NGS_HOST_GRAMS", cls=ssl.StringIndex, **kw):
    if host:
        os.environ[env] = "1"
    try:
        return cls(words, rs, wts, **kw)
    finally:
        os.environ.pop(env, None)


def _corpora():
    rng = random.Random(7)
    words, wts, _ = ssl.synth.gen_corpus(20000, seed=5)
    yield "synth", words, 1, wts
    yield "acgt", [bytes(rng.choice(b"ACGT") for _ in range(rng.randint(6, 40))) for _ in range(30000)], 1, None
    yield "repeats", [b"AAAAAAAAAA", b"ABABABABAB", b"XYZXYZXYZ", b"abcabcabcabc"] * 50 + [b"AB", b"A"], 1, None
    mixed, _, _ = ssl.synth.gen_corpus(5000, seed=8, min_len=1, span=12, row_size=2)
    yield "mixed", mixed, 2, None
    yield "short_only", [b"AB", b"CD", b"EFG", b"HIJK"], 1, None


@pytest.mark.parametrize("name,words,rs,wts", list(_corpora()), ids=lambda x: x if isinstance(x, str) else "")
def test_gpu_build_matches_host_build(name, words, rs, wts):
    g = _build(words, rs, wts)
    h = _build(words, rs, wts, host=True)
    dg, dh = _digest(g), _digest(h)
    assert dg == dh, f"{name}: device build {dg} vs host build {dh}"
    assert g.lib_size() == h.lib_size() and g.size() == h.size()
    qs = [w for w in words if w][:200:3] + [b"ACGTACGTAC", b"ABAB", b"zzzz"]
    for thr, limit in [(0.3, 100), (0.0, 20)]:
        assert g.score_batch(qs, thr, limit) == h.score_batch(qs, thr, limit)
    if name == "acgt":
        assert dg[2] > 256, "dense lists should take more than 256 skip buckets"
    g.dispose()
    h.dispose()


def _messy(rng, n, rs, alpha="ABCDEFabcdef0123 .-_#\t"):
    words = []
    for i in range(n * rs):
        r = rng.random()
        if r < 0.04:
            words.append(None)
        elif r < 0.07:
            words.append("  \t ")  # blank: as a row head the row yields nothing
        elif r < 0.2 and words:
            words.append(rng.choice([w for w in words[-50:] if w is not None] or ["X"]))  # repeats
        else:
            words.append("".join(rng.choice(alpha) for _ in range(rng.randint(1, 14))))
    wts = [rng.choice([1.0, 0.5, 2.0, 0.0, -0.0, -0.5, 0.75, 3.0]) for _ in words]
    return words, wts


@pytest.mark.parametrize("rs,weighted,wide", [(1, True, False), (3, True, False), (2, False, False),
                                              (4, True, True), (1, False, True)])
def test_gpu_intern_matches_host_intern(rs, weighted, wide):
    rng = random.Random(rs * 31 + weighted * 7 + wide)
    words, wts = _messy(rng, 6000, rs)
    if not weighted:
        wts = None
    cls = ssl.WideStringIndex if wide else ssl.StringIndex
    if not wide:
        words = [None if w is None else w.encode("latin-1") for w in words]
    kw = {"gram_size": 2} if wide else {}
    g = _build(words, rs, wts, cls=cls, **kw)
    h = _build(words, rs, wts, host=True, env="NGS_HOST_INTERN", cls=cls, **kw)
    dg, dh = _digest(g), _digest(h)
    assert dg == dh, f"rs={rs} weighted={weighted} wide={wide}: device {dg} vs host {dh}"
    assert g.size() == h.size() and g.lib_size() == h.lib_size() and g.num_keys() == h.num_keys()
    qs = [w for w in words if w][:300:7] + (["*", ""] if wide else [b"*", b""])
    for thr, limit in [(0.3, 100), (0.0, 7)]:
        assert g.score_batch(qs, thr, limit) == h.score_batch(qs, thr, limit)
    g.dispose()
    h.dispose()
