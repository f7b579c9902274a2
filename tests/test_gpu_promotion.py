"""Exact-match promotion next to large weights on the GPU, exact against the oracle (GPU).

A promoted key is the score 100 (nGramSearch.hpp:326-337 through ScoreComparer,
nGramSearch.h:262-269): w*s = 150 ranks above it, w*s = 100 ties with it and the shorter key
goes first, and a promoted key's own w*s above 100 is lowered to 100. calcScore merges the
short scores before the long ones (hpp:393-394), so a short alias above 100 of a key that a long
term promotes is overwritten (key_promoted_long). The oracle, which the reference itself pins
on these semantics (tests/test_ref_fuzz.py, golden promotion*.json), is matched exactly on every
tier: the lean and full wave kernels (limits <= 128), tier 2 (limit 500), the general path
(queries of <= 3 characters, limit 1500), the rank-list path (one weight <= 200) and the server
kernel.
"""
import random
import zlib

import pytest

from oracle_py import OracleIndex
from tiecheck import bits

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu
POOL = [1.0, 100.0, 150.0, 1000.0, 0.0, -1.0, 0.5, 2.0]


def assert_exact(ours, ref, where):
    assert len(ours) == len(ref), f"{where}: {len(ours)} results vs oracle {len(ref)}\n{ours[:6]}\n{ref[:6]}"
    for i, ((k1, s1), (k2, s2)) in enumerate(zip(ours, ref)):
        assert k1 == k2 and bits(s1) == bits(s2), f"{where}: #{i} {k1!r}|{s1!r} vs oracle {k2!r}|{s2!r}"


def _small_corpus(rng):
    alpha = "ABCDE" if rng.random() < 0.5 else "ABCDEFGH XY"
    row = rng.choice([1, 1, 2, 3])
    words, weights, keys = [], [], []
    for _ in range(rng.randint(3, 14)):
        for j in range(row):
            r = rng.random()
            if j == 0 and keys and r < 0.15:
                w = rng.choice(keys)
            elif r < 0.25:
                w = "".join(rng.choice(alpha) for _ in range(rng.randint(1, 5)))
            else:
                w = "".join(rng.choice(alpha) for _ in range(rng.randint(6, 12)))
            if rng.random() < 0.15:
                w = w.lower()
            if j == 0:
                keys.append(w)
            words.append(w.encode())
            weights.append(rng.choice(POOL))
    return words, row, weights, keys


def _small_queries(rng, words, keys, n):
    out = []
    for _ in range(n):
        r = rng.random()
        src = rng.choice(keys).encode()
        if r < 0.45:
            q = src
        elif r < 0.55:
            q = src.lower()
        elif r < 0.8:
            w = rng.choice(words)
            a = rng.randrange(len(w))
            q = w[a:a + rng.randint(1, 9)]
        else:
            w = bytearray(rng.choice(words))
            w[rng.randrange(len(w))] = ord(rng.choice("ABCDEXYZ"))
            q = bytes(w)
        out.append(q or b"A")
    return out


def test_promotion_small_corpora():
    """The fuzz of test_ref_fuzz.py on the GPU: 120 small corpora, every limit tier."""
    rng = random.Random(7100)
    for c in range(120):
        words, row, weights, keys = _small_corpus(rng)
        gi = ssl.StringIndex(words, row, weights)
        oi = OracleIndex(words, row, weights)
        qs = _small_queries(rng, words, keys, 12)
        for thr in (0.0, 0.3):
            for limit in (1, 3, 100, 500, 1500, 0):
                got = gi.score_batch(qs, thr, limit)
                for q, g in zip(qs, got):
                    assert_exact(g, oi.score(q, thr, limit), f"corpus {c} {words} w={weights} q={q!r} thr={thr} "
                                                             f"limit={limit}")
        for q in qs[:4]:  # single queries: the latency path and, after a few calls, the server kernel
            assert_exact(gi.score(q, 0.0, 100), oi.score(q, 0.0, 100), f"corpus {c} single q={q!r}")
        gi.dispose()
        oi.close()


@pytest.mark.parametrize("kind", ["pool_rows1", "pool_rows3", "uniform150", "uniform1000"])
def test_promotion_synthetic(kind):
    """Synthetic libraries of 20k rows: weights from the pool (rowSize 1 and 3, aliases), or one
    weight of 150 (rank lists at threshold 0) or 1000 (no rank lists: w * fl(1/n) can pass 100)."""
    rng = random.Random(zlib.crc32(kind.encode()))
    row = 3 if kind == "pool_rows3" else 1
    words, _, srng = ssl.synth.gen_corpus(20000, seed=31, row_size=row, min_len=4 if row == 3 else 8)
    if kind.startswith("pool"):
        weights = [rng.choice(POOL) for _ in words]
    else:
        weights = [float(kind[len("uniform"):])] * len(words)
    gi = ssl.StringIndex(words, row, weights)
    oi = OracleIndex(words, row, weights)
    keys = [words[i] for i in range(0, len(words), row)]
    qs = ssl.synth.gen_queries(words, row, 150, srng)
    qs += [rng.choice(keys) for _ in range(60)] + [rng.choice(keys).lower() for _ in range(20)]
    qs += [rng.choice(keys)[:rng.randint(2, 8)] for _ in range(40)]
    for thr, limit in [(0.0, 100), (0.3, 100), (0.0, 3), (0.5, 1), (0.0, 500), (0.2, 0)]:
        got = gi.score_batch(qs, thr, limit)
        for q, g in zip(qs, got):
            assert_exact(g, oi.score(q, thr, limit), f"{kind} q={q!r} thr={thr} limit={limit}")
    gi.dispose()
