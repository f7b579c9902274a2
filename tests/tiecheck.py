"""Tie-aware comparison against the reference's answers (SURVEY.md §0.5, §7 "Hard parts").

The reference orders results by score desc, then key length asc (ScoreComparer,
nGramSearch.h:262-269) through std::partial_sort over unordered_map order
(nGramSearch.hpp:397-401), so the order INSIDE an equal (score, length) group is
unspecified and even changes with `limit`. An answer is accepted iff
  1. it has exactly as many results as the reference at the same limit;
  2. every returned key is in the reference's full (limit=0) answer with the same fp32 bits
     (+0.0 and -0.0 compare equal: the sign of a zero max is iteration-order dependent);
  3. it is sorted by (score desc, length asc);
  4. its multiset of (score, length) equals that of the first `limit` of the full answer,
     i.e. strictly better groups are identical and the cut group is a valid subset.
"""
from __future__ import annotations

import struct


def bits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def f32(b: int) -> float:
    return struct.unpack("<f", struct.pack("<I", b))[0]


def canon(b: int) -> int:
    return 0 if b == 0x80000000 else b


def check(ours, ref_n: int, full_keys, full_score_bits, where: str = "") -> None:
    """ours: list of (key bytes/str, score float or bits int)."""
    def kb(k):
        return k if isinstance(k, bytes) else k.encode("latin-1")

    def sb(s):
        return canon(s if isinstance(s, int) else bits(s))

    ours = [(kb(k), sb(s)) for k, s in ours]
    full = [(kb(k), canon(s)) for k, s in zip(full_keys, full_score_bits)]
    assert len(ours) == ref_n, f"{where}: count {len(ours)} != reference {ref_n}"
    ref_score = dict(full)
    assert len(ref_score) == len(full), f"{where}: duplicate key in reference answer"
    seen = set()
    for k, s in ours:
        assert k not in seen, f"{where}: key {k!r} returned twice"
        seen.add(k)
        assert k in ref_score, f"{where}: key {k!r} not in reference answer"
        assert ref_score[k] == s, f"{where}: key {k!r} score {f32(s)!r} != reference {f32(ref_score[k])!r}"
    for (k1, s1), (k2, s2) in zip(ours, ours[1:]):
        a, b = f32(s1), f32(s2)
        assert a > b or (a == b and len(k1) <= len(k2)), f"{where}: order violated at {k1!r} / {k2!r}"
    mine = sorted((s, len(k)) for k, s in ours)
    theirs = sorted((s, len(k)) for k, s in full[:ref_n])
    assert mine == theirs, f"{where}: (score, length) groups differ from the reference's top-{ref_n}"
