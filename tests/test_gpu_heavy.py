"""Heavy queries (match-count threshold cmin 2) through the lean kernel's spill path, exact vs the
oracle. At cmin 2 every term sharing a 4-gram with the query survives: the survivors overflow the
LDS survivor list and spill to HBM for k_emit (up to kEmitCap = 1024 per query), and above that
the query is handed over to tier 1b. Both corpora use 8-character queries (6 grams, thr 0.3 ->
cmin 2), as in nGramSearch.hpp:278-301 + 310-341."""
import random

import pytest

from oracle_py import OracleIndex
from tiecheck import bits

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu


def _words(rng, alphabet, n, lo, hi):
    return [bytes(rng.choice(alphabet) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def _queries(rng, words, n, qlen=8):
    out = []
    for _ in range(n):
        src = rng.choice([w for w in words if len(w) >= qlen])
        o = rng.randrange(len(src) - qlen + 1)
        q = bytearray(src[o:o + qlen])
        q[rng.randrange(qlen)] = src[0]
        out.append(bytes(q))
    return out


@pytest.mark.parametrize("alphabet,rows,lo,hi,expect_handover", [
    (b"ABCDEFGHIJKL", 60000, 10, 30, False),  # a few hundred survivors: spilled, scored by k_emit
    (b"ABCDEFGH", 40000, 6, 30, True),         # thousands: beyond kEmitCap, tier 1b
])
def test_cmin2_spill_parity(alphabet, rows, lo, hi, expect_handover):
    rng = random.Random(rows + len(alphabet))
    words = _words(rng, alphabet, rows, lo, hi)
    wts = [0.5 + rng.random() / 2 for _ in words]
    gi = ssl.StringIndex(words, 1, wts)
    gi.set_timing(True)  # ngsLastStats
    oi = OracleIndex(words, 1, wts)
    qs = _queries(rng, words, 40)
    for thr, limit in [(0.3, 100), (0.3, 7)]:
        got = gi.score_batch(qs, thr, limit)
        st = gi.last_stats()
        for q, g in zip(qs, got):
            ref = oi.score(q, thr, limit)
            assert len(g) == len(ref), f"q={q!r} thr={thr} limit={limit}: {len(g)} vs {len(ref)}"
            for i, ((k1, s1), (k2, s2)) in enumerate(zip(g, ref)):
                assert k1 == k2 and bits(s1) == bits(s2), f"q={q!r} #{i}: {k1!r}|{s1} vs {k2!r}|{s2}"
        if expect_handover:
            assert st["handover_queries"] > 0, st
        else:  # most finish in the lean kernel (a part with > 64 sketch candidates hands over)
            assert st["handover_queries"] < len(qs) // 4 and st["survivors"] / len(qs) > 128, st
    # a heavy list longer than the side launches' grids (4096): grid-stride in every stage
    small = gi.score_batch(qs, 0.3, 100)
    big = gi.score_batch(qs * 128, 0.3, 100)
    for i, g in enumerate(big):
        assert g == small[i % len(qs)], f"batch of {len(big)}: q#{i} differs"
    gi.dispose()


@pytest.mark.parametrize("alphabet,rows,lo,hi,qlen", [
    (b"ABCDEFGHIJKLMNOPQRSTUVWXYZ", 60000, 8, 24, 12),  # hundreds of one-hit terms: part_ones
    (b"ABCDEFGHIJKL", 30000, 3, 20, 10),                # thousands, with a shortLib beside
])
def test_cmin1_ones_and_short_routing(alphabet, rows, lo, hi, qlen):
    """Threshold 0 (cmin 1): the heavy list's lean launch counts the parts with part_ones (one-hit
    terms straight to the survivor slots, the rest resolved exactly); queries with more than
    kEmitCap survivors hand over to tier 1b. Short queries (|q| < 9 with a shortLib) take the full
    list into tier 1b. Exact vs the oracle."""
    rng = random.Random(rows + qlen)
    words = _words(rng, alphabet, rows, lo, hi)
    wts = [rng.choice([1.0, 0.5, 0.25 + rng.random()]) for _ in words]
    gi = ssl.StringIndex(words, 1, wts)
    gi.set_timing(True)
    oi = OracleIndex(words, 1, wts)
    cases = [(_queries(rng, words, 40, qlen), 0.0, "ones")]
    if lo < 6:
        cases.append((_queries(rng, words, 24, 6), 0.3, "short"))
    for qs, thr, kind in cases:
        for limit in (100, 10):
            got = gi.score_batch(qs, thr, limit)
            st = gi.last_stats()
            for q, g in zip(qs, got):
                ref = oi.score(q, thr, limit)
                assert len(g) == len(ref), f"{kind} q={q!r} limit={limit}: {len(g)} vs {len(ref)}"
                for i, ((k1, s1), (k2, s2)) in enumerate(zip(g, ref)):
                    assert k1 == k2 and bits(s1) == bits(s2), f"{kind} q={q!r} #{i}: {k1!r}|{s1} vs {k2!r}|{s2}"
            if kind == "ones":
                assert st["heavy_queries"] == len(qs) and st["full_queries"] == 0, st
            else:
                assert st["full_queries"] == len(qs), st
    gi.dispose()


def _digest_flags(gi):
    import ctypes as C
    from stringsearchlib_amd import _native
    out = (C.c_uint64 * 17)()
    assert _native.lib().ngsIndexDigest(gi.handle, out, 17) == 17
    return out[16]


@pytest.mark.parametrize("weight", [None, 0.5, 2.5, -2.0, 1e-45])  # (weight 0 drops a row, hpp:144)
@pytest.mark.parametrize("alphabet,rows,lo,hi,qlen", [
    (b"ABCDEFGHIJKLMNOPQRSTUVWXYZ", 60000, 8, 24, 12),  # C2's shape: thousands of one-hit terms
    (b"ABC", 20000, 6, 20, 10),                          # repeated grams in every query and key
])
def test_cmin1_rank_lists(alphabet, rows, lo, hi, qlen, weight):
    """Threshold 0 on an index with one weight (NULL weights: 1.0), one pair per term and one term
    per key: tier 1a counts only the multi-hit terms (cmin 2) and k_emit takes the one-hit records
    from the first `limit` key ranks of each list (DevIndex.rank_post, emit_rank_prefix). Exact vs the
    oracle and vs the same index without rank lists (NGS_NO_RANK_LISTS, part_ones), for weights that
    make every count tie (negative, a subnormal that underflows) as well as ordinary ones."""
    import os
    rng = random.Random(rows + qlen + len(alphabet))
    words = list(dict.fromkeys(_words(rng, alphabet, rows, lo, hi)))  # one term per key
    wts = None if weight is None else [weight] * len(words)
    gi = ssl.StringIndex(words, 1, wts)
    os.environ["NGS_NO_RANK_LISTS"] = "1"
    try:
        gp = ssl.StringIndex(words, 1, wts)
    finally:
        del os.environ["NGS_NO_RANK_LISTS"]
    assert _digest_flags(gi) & 8 and not _digest_flags(gp) & 8
    gi.set_timing(True)
    gp.set_timing(True)
    oi = OracleIndex(words, 1, wts)
    qs = _queries(rng, words, 48, qlen) + [b"ABCABCABCABC", b"AAAAAAAAAAAA", b"ZZZZZZZZZZZZ"]
    for limit in (100, 10, 1, 128):
        got = gi.score_batch(qs, 0.0, limit)
        st = gi.last_stats()
        plain = gp.score_batch(qs, 0.0, limit)
        stp = gp.last_stats()
        for q, g, p in zip(qs, got, plain):
            ref = oi.score(q, 0.0, limit)
            assert len(g) == len(ref), f"q={q!r} limit={limit}: {len(g)} vs {len(ref)}"
            for i, ((k1, s1), (k2, s2)) in enumerate(zip(g, ref)):
                assert k1 == k2 and bits(s1) == bits(s2), f"q={q!r} limit={limit} #{i}: {k1!r}|{s1} vs {k2!r}|{s2}"
            assert g == p, f"q={q!r} limit={limit}: rank lists differ from part_ones"
        if len(alphabet) > 3:  # the multi-hit terms only reach the survivor slots
            assert st["survivors"] * 4 < stp["survivors"], (st, stp)
    gi.dispose()
    gp.dispose()
