"""Degenerate arguments of the reference ABI on the GPU, exact against the oracle (GPU).

The reference takes the threshold and the limit as given: `s < threshold` skips a term
(nGramSearch.hpp:315), so a NaN or negative threshold skips nothing and one above 1 keeps only what
reaches it (short-search scores, promoted exact matches); `limit` is a uint32, 0 meaning every
result (hpp:399-401, 420-425). tests/test_ref_fuzz.py::test_oracle_vs_reference_degenerate_args
pins the oracle on these against the compiled reference; here every path of the library answers
them exactly like the oracle: scoreBatch over large batches (tier 1a, heavy list, tier 1b, tier 2,
the general path), batches of <= 16 queries (the latency path), single score()/search() calls, and
the server kernel (ngsServe).
"""
import math
import random

import pytest

from oracle_py import OracleIndex
from tiecheck import bits

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu

THRESHOLDS = [-1.0, float("nan"), 1.0, 1.5, 0.999, 1.0 / 3.0, 0.7]
LIMITS = [1, 100, 2**31, 2**32 - 1, 0]
POOL = [1.0, 100.0, 150.0, 0.5, 2.0, 0.0, -1.0]


def assert_exact(ours, ref, where):
    assert len(ours) == len(ref), f"{where}: {len(ours)} results vs oracle {len(ref)}\n{ours[:6]}\n{ref[:6]}"
    for i, ((k1, s1), (k2, s2)) in enumerate(zip(ours, ref)):
        assert k1 == k2 and bits(s1) == bits(s2), f"{where}: #{i} {k1!r}|{s1!r} vs oracle {k2!r}|{s2!r}"


def _tag(thr):
    return "nan" if math.isnan(thr) else repr(thr)


@pytest.fixture(scope="module")
def corpus():
    rng = random.Random(61019)
    words, _, srng = ssl.synth.gen_corpus(20000, seed=61, row_size=1, min_len=4)
    weights = [rng.choice(POOL) for _ in words]
    qs = ssl.synth.gen_queries(words, 1, 200, srng)
    qs += [rng.choice(words) for _ in range(40)] + [rng.choice(words).lower() for _ in range(10)]
    qs += [rng.choice(words)[:rng.randint(1, 8)] for _ in range(30)] + [b"", b"*"]
    gi = ssl.StringIndex(words, 1, weights)
    oi = OracleIndex(words, 1, weights)
    yield words, weights, qs, gi, oi
    gi.dispose()
    oi.close()


@pytest.mark.parametrize("thr", THRESHOLDS, ids=_tag)
def test_degenerate_batches(corpus, thr):
    """scoreBatch over the whole query set (the batch path) and over 12 queries (the latency path)."""
    _, _, qs, gi, oi = corpus
    for limit in LIMITS:
        refs = [oi.score(q, thr, limit) for q in qs]
        got = gi.score_batch(qs, thr, limit)
        for q, g, r in zip(qs, got, refs):
            assert_exact(g, r, f"batch q={q!r} thr={_tag(thr)} limit={limit}")
        if limit >= 2**31:  # a limit past every key is "all of them", as 0
            assert [len(g) for g in got] == [len(g) for g in gi.score_batch(qs, thr, 0)]
        few = qs[::25][:12]
        for q, g in zip(few, gi.score_batch(few, thr, limit)):
            assert_exact(g, oi.score(q, thr, limit), f"latency q={q!r} thr={_tag(thr)} limit={limit}")


@pytest.mark.parametrize("thr", THRESHOLDS, ids=_tag)
def test_degenerate_single_and_server(corpus, thr):
    """score()/search() one query at a time, on the launch path and through the server kernel."""
    words, weights, qs, _, oi = corpus
    sample = qs[::17]
    for serve in (False, True):
        gi = ssl.StringIndex(words, 1, weights)
        try:
            gi.serve(serve)
            for limit in (1, 100, 2**32 - 1):
                for q in sample:
                    ref = oi.score(q, thr, limit)
                    assert_exact(gi.score(q, thr, limit), ref, f"score serve={serve} q={q!r} thr={_tag(thr)} "
                                                               f"limit={limit}")
                    assert gi.search(q, thr, limit) == [k for k, _ in ref]
                if serve and limit == 1 and thr > 0:
                    # a long query after the sample: the server kernel answers it (at thresholds <= 0 or
                    # NaN every term with a shared gram survives, cmin 1: the server hands such queries
                    # to the regular path, which stops it)
                    q = next(w for w in words if len(w) >= 12)
                    assert_exact(gi.score(q, thr, 1), oi.score(q, thr, 1), f"served q={q!r} thr={_tag(thr)}")
                    assert gi.serve_state() == 2
        finally:
            gi.dispose()
