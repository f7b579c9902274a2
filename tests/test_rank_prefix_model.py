"""CPU model of the threshold-0 rank-list shortcut (DevIndex.rank_post; ngs_kernels.hip
emit_rank_prefix), checked by brute force against the reference's ordering.

At threshold 0 a term survives with one hit. When every (term, key) pair has the same weight, every
term has one pair and every key one term, a term's record is (score of its hit count, key rank)
(calcScore nGramSearch.hpp:318-336 with fp32 max(w*s, 0); ScoreComparer nGramSearch.h:249-270:
score desc, then key rank asc). The kernel counts only the multi-hit terms, takes their top L, and
merges the first L key ranks of each of the query's gram lists as one-hit records, dropping an entry
whose key is among the multi-hit top L and any record not below the running L-th (tau). This model
does exactly that, in plain Python with fp32 rounding, and compares it with the full sort of every
survivor over random corpora, limits and weights (ties included: 0-score and subnormal weights)."""
import random
import struct

import pytest


def f32(x: float) -> float:
    return struct.unpack("f", struct.pack("f", x))[0]


def enc(w: float, s: float) -> int:
    sc = f32(f32(w) * s)
    return (struct.unpack("I", struct.pack("f", sc))[0] + 1) if sc > 0 else 1


def record(w, n, key, count):  # ascending order = reference order
    return ((~enc(w, f32(count / n))) & 0xFFFFFFFF, key)


def model(lists, grams, w, L):
    n = len(grams)
    cnt = {}
    for g in grams:  # searchLong with multiplicity (nGramSearch.hpp:278-301)
        for k in lists.get(g, ()):
            cnt[k] = cnt.get(k, 0) + 1
    truth = sorted(record(w, n, k, c) for k, c in cnt.items())[:L]
    multi = sorted(record(w, n, k, c) for k, c in cnt.items() if c >= 2)[:L]
    kset = {k for _, k in multi}
    tau = multi[L - 1] if len(multi) >= L else None
    cand = list(multi)
    for g in grams:  # each occurrence's list, its first L key ranks
        for k in sorted(lists.get(g, ()))[:L]:
            r = record(w, n, k, 1)
            if tau is not None and not r < tau:
                break  # ascending ranks: the rest of this list is worse too
            if k in kset:
                continue
            cand.append(r)
        # (the kernel also trims the buffer and lowers tau as it goes; that only drops more
        # records that cannot enter the top L)
    assert len({k for _, k in cand}) == len(cand), "a key twice in the buffer"
    return sorted(cand)[:L], truth


@pytest.mark.parametrize("seed", range(6))
def test_rank_prefix_matches_full_sort(seed):
    rng = random.Random(seed)
    for _ in range(60):
        alpha = rng.choice(["ABC", "ABCDEFGH", "ABCDEFGHIJKLMNOP"])
        words = list(dict.fromkeys("".join(rng.choice(alpha) for _ in range(rng.randint(6, 14)))
                                   for _ in range(rng.randint(50, 300))))
        w = rng.choice([1.0, 0.5, 2.5, -2.0, 1e-45])
        lists = {}
        for key, t in enumerate(words):  # key rank = position (one term per key)
            for i in range(len(t) - 2):
                lists.setdefault(t[i:i + 3], set()).add(key)
        q = "".join(rng.choice(alpha) for _ in range(rng.randint(4, 12)))
        grams = [q[i:i + 3] for i in range(len(q) - 2)]
        L = rng.choice([1, 3, 10, 100])
        got, truth = model(lists, grams, w, L)
        assert got == truth, (q, w, L)
