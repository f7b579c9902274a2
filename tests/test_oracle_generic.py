"""The gram-size / UTF-32 restatement (oracle/ngs_oracle_g.c) — the checker of the indexG /
indexW extensions, which the reference does not have (parity unpinned).

It is pinned as far as it can be:
* g = 3 on byte strings it must answer EXACTLY like the pinned narrow oracle (keys, order,
  fp32 bits), on every golden fixture (and tie-aware like the reference itself) and on
  seeded random corpora — the two restatements share no code;
* UTF-32 input that is ASCII must answer like the byte path;
* small hand-computed answers for g = 1, 2 and non-ASCII text anchor the scaled thresholds
  (DESIGN.md §9).
"""
import random
import struct

import pytest

from conftest import fixture_weights, fixture_words, load_fixtures
from oracle_py import OracleIndex, OracleIndexG
from tiecheck import bits, check

import stringsearchlib_amd as ssl

FIXTURES = load_fixtures()


def f32(b):
    return struct.unpack("<f", struct.pack("<I", b))[0]


def same(a, b, where):
    assert len(a) == len(b), f"{where}: {len(a)} vs {len(b)}\n{a[:5]}\n{b[:5]}"
    for i, ((k1, s1), (k2, s2)) in enumerate(zip(a, b)):
        assert k1 == k2 and bits(s1) == bits(s2), f"{where}: #{i} {k1!r}|{s1!r} vs {k2!r}|{s2!r}"


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_generic_g3_equals_pinned_oracle_on_fixtures(fx):
    words, weights = fixture_words(fx), fixture_weights(fx)
    gx = OracleIndexG(words, fx["rowSize"], weights, g=3)
    ox = OracleIndex(words, fx["rowSize"], weights)
    assert gx.size() == ox.size() == fx["size"]
    assert gx.lib_size() == ox.lib_size() == fx["libSize"]
    for pi, ph in enumerate(fx["phases"]):
        if ph["validChar"] is not None:
            gx.set_valid_char(ph["validChar"].encode("latin-1"))
            ox.set_valid_char(ph["validChar"].encode("latin-1"))
        for ci, c in enumerate(ph["cases"]):
            q, thr, limit = c["q"].encode("latin-1"), f32(c["thr"]), c["limit"]
            where = f"{fx['name']}[{pi}.{ci}] q={q!r}"
            ours = gx.score(q, thr, limit)
            check(ours, len(c["keys"]), c["full_keys"], c["full_scores"], where)
            same(ours, ox.score(q, thr, limit), where)


def _queries(rng, keys, n):
    alpha = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 abcxyz-#.%$@*\t"
    out = []
    for i in range(n):
        src = rng.choice(keys)
        kind = i % 5
        if kind == 0:
            l = min(12, len(src)); o = rng.randrange(len(src) - l + 1)
            q = bytearray(src[o:o + l]); q[rng.randrange(l)] = rng.choice(alpha[:26]); q = bytes(q)
        elif kind == 1:
            l = rng.randint(1, min(8, len(src))); o = rng.randrange(len(src) - l + 1); q = src[o:o + l]
        elif kind == 2:
            q = src if rng.random() < 0.5 else src.lower()
        elif kind == 3:
            q = bytes(rng.choice(alpha) for _ in range(rng.randint(0, 20)))
        else:
            q = b"  " + src.replace(b" ", b"-") + b"!! "
        out.append(q)
    return out + [b"", b"*", b"   ", b"A", b"AB"]


@pytest.mark.parametrize("seed", [1, 2])
def test_generic_g3_equals_pinned_oracle_random(seed):
    rng = random.Random(seed)
    words, wts, _ = ssl.synth.gen_corpus(1500, seed=seed, min_len=1, span=20, row_size=2)
    gx, ox = OracleIndexG(words, 2, wts, g=3), OracleIndex(words, 2, wts)
    assert gx.size() == ox.size() and gx.lib_size() == ox.lib_size()
    for q in _queries(rng, [w for w in words if w], 80):
        for thr, limit in [(0.0, 100), (0.3, 10), (0.0, 0)]:
            same(gx.score(q, thr, limit), ox.score(q, thr, limit), f"seed={seed} q={q!r}")


@pytest.mark.parametrize("g", [1, 2, 3])
def test_wide_ascii_equals_narrow(g):
    rng = random.Random(10 + g)
    words, wts, _ = ssl.synth.gen_corpus(800, seed=g, min_len=1, span=14)
    nx = OracleIndexG(words, 1, wts, g=g)
    wx = OracleIndexG([w.decode() for w in words], 1, wts, g=g, wide=True)
    assert nx.size() == wx.size() and nx.lib_size() == wx.lib_size()
    for q in _queries(rng, words, 60):
        n = [(k.decode(), s) for k, s in nx.score(q, 0.0, 50)]
        same(wx.score(q.decode(), 0.0, 50), n, f"g={g} q={q!r}")


def test_known_answers_g2():
    # terms of >= 4 characters are gram-indexed; "HELP": grams HE EL LP, HELLO holds 2 of 3
    ix = OracleIndexG([b"HELLO", b"WORLD"], 1, None, g=2)
    assert ix.size() == 2 and ix.lib_size() == 8
    assert ix.score(b"hello") == [(b"HELLO", 100.0)]
    assert ix.score(b"HELP") == [(b"HELLO", struct.unpack("<f", struct.pack("<f", 2 / 3))[0])]


def test_known_answers_g1():
    # g = 1: every term of >= 2 characters is long; a 2-character query has 2 unigrams and
    # runs the short search too (|q| < 3) over the (empty) shortLib
    ix = OracleIndexG([b"AB", b"BA", b"ABC", b"Z"], 1, None, g=1)
    assert ix.size() == 4 and ix.lib_size() == 3
    # threshold 0 keeps zero scores: Z is scored 0 by the short search
    assert ix.score(b"AB") == [(b"AB", 100.0), (b"BA", 1.0), (b"ABC", 1.0), (b"Z", 0.0)]
    # |q| <= g: the short search scans the whole library (hpp:247), Z included
    assert ix.score(b"Z", 0.5) == [(b"Z", 100.0)]
    assert ix.score(b"A", 0.5) == [(b"AB", 1.0), (b"BA", 1.0), (b"ABC", 1.0)]


def test_known_answers_wide_g2():
    ix = OracleIndexG(["日本語テキスト", "日本"], 1, None, g=2, wide=True)
    # short search (|q| = 3 < 6) over shortLib {日本}: distance 1 -> 2/3; gram search: 日本, 本語
    two_thirds = struct.unpack("<f", struct.pack("<f", 2 / 3))[0]
    assert ix.score("日本語") == [("日本語テキスト", 1.0), ("日本", two_thirds)]
    # lower-case ASCII folds, other code points are kept as they are; promotion compares the
    # key without case folding (hpp:330-334), so only an upper-case key is promoted
    ix2 = OracleIndexG(["straße", "STRASSE", "ÖL STRAßE"], 1, None, g=2, wide=True)
    three_fifths = struct.unpack("<f", struct.pack("<f", 3 / 5))[0]
    assert ix2.score("STRAßE", 0.5) == [("straße", 1.0), ("ÖL STRAßE", 1.0), ("STRASSE", three_fifths)]
    assert ix2.score("öl straße", 0.9) == []  # ö is not folded: no 'ÖL' gram in "öl"
    assert ix2.score("Öl straße", 0.9) == [("ÖL STRAßE", 100.0)]
    assert ix2.size() == 3


def test_wide_invalid_code_units_are_spaces():
    # values above 0x10FFFF are not code points: escaped to spaces like invalid bytes
    ix = OracleIndexG(["KEY1", [0x41, 0x42, 0x43, 0x44, 0x110000, 0x45]], 2, None, g=2, wide=True)
    assert ix.score("abcd e") == [("KEY1", 1.0)]
    assert ix.score([0x61, 0x62, 0x63, 0x64, 0xFFFFFFFF, 0x65]) == [("KEY1", 1.0)]
