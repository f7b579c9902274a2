"""GPU path of the indexG / indexW extensions against the gram-size / UTF-32 restatement
(oracle/ngs_oracle_g.c; parity unpinned beyond g = 3 bytes — see test_oracle_generic.py for
how that restatement is tied to the pinned one).

Exact comparisons (keys, order, fp32 bits) on seeded corpora with non-ASCII code points
(Latin-1, CJK, astral), aliases, NULL holes, zero / negative weights, invalid code units,
g = 1, 2, 3, every query-length regime (full scan, short search, wave kernel, general path),
plus: wide g = 3 on ASCII == the narrow (reference) path, width-mismatched calls answer 0,
the device API on a wide index.
"""
import random
import struct
import zlib

import pytest

from oracle_py import OracleIndexG
from tiecheck import bits

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu

WIDE_ALPHA = ("ABCDEFGHIJKLMNOP" "abcdxyz" "0123456789" "  " "éßÖçñ" "日本語中文字" "テキスト"
              "\U0001F600\U00020000")


def assert_exact(ours, ref, where):
    assert len(ours) == len(ref), f"{where}: {len(ours)} results vs oracle {len(ref)}\n{ours[:5]}\n{ref[:5]}"
    for i, ((k1, s1), (k2, s2)) in enumerate(zip(ours, ref)):
        assert k1 == k2 and bits(s1) == bits(s2), f"{where}: #{i} {k1!r}|{s1!r} vs oracle {k2!r}|{s2!r}"


def wide_corpus(rng, rows, row_size, lo=1, hi=24, alpha=WIDE_ALPHA):
    words = []
    for _ in range(rows * row_size):
        n = rng.randint(lo, hi)
        words.append("".join(rng.choice(alpha) for _ in range(n)))
    return words


def wide_queries(rng, keys, n):
    out = []
    for i in range(n):
        src = rng.choice(keys)
        kind = i % 8
        if kind == 0:      # window with one substitution
            l = min(12, len(src)); o = rng.randrange(len(src) - l + 1)
            q = list(src[o:o + l]); q[rng.randrange(l)] = rng.choice(WIDE_ALPHA); q = "".join(q)
        elif kind == 1:    # short substring
            l = rng.randint(1, min(8, len(src))); o = rng.randrange(len(src) - l + 1); q = src[o:o + l]
        elif kind == 2:    # exact key, maybe lower-cased
            q = src if rng.random() < 0.5 else src.lower()
        elif kind == 3:    # junk, with code units that are not code points
            q = [rng.choice([ord(rng.choice(WIDE_ALPHA)), 0x110000, 0xFFFFFFFF, 0x7F, ord("-")])
                 for _ in range(rng.randint(0, 16))]
        elif kind == 4:    # two keys glued
            q = src + " " + rng.choice(keys)
        elif kind == 5:    # padded / escaped
            q = "  " + src.replace(" ", "-") + "!! "
        elif kind == 6:    # long query: more grams than the wave kernel takes
            q = (src + " ") * (90 // (len(src) + 1) + 1)
        else:
            l = min(len(src), rng.randint(6, 20)); o = rng.randrange(len(src) - l + 1); q = src[o:o + l]
        out.append(q)
    return out + ["", "*", "   ", "日", "日本"]


def _shape(words, rng):
    words = list(words)
    for i in range(0, len(words), 37):
        words[i] = None
    wts = [rng.choice([1.0, 0.5, 2.0, 0.0, -0.5, 0.75]) for _ in words]
    return words, wts


@pytest.mark.parametrize("g", [1, 2, 3])
def test_wide_parity_vs_generic_oracle(g):
    rng = random.Random(zlib.crc32(f"wide{g}".encode()))
    words, wts = _shape(wide_corpus(rng, 2500, 2), rng)
    gi = ssl.WideStringIndex(words, 2, wts, gram_size=g)
    oi = OracleIndexG(words, 2, wts, g=g, wide=True)
    assert gi.size() == oi.size() and gi.lib_size() == oi.lib_size()
    assert gi.gram_size() == g
    keys = [w for w in words[::2] if w and w.strip()]
    qs = wide_queries(rng, keys, 96)
    for thr, limit in [(0.0, 100), (0.3, 100), (0.5, 7), (0.0, 0), (1.0, 5), (0.0, 1500)]:
        got = gi.score_batch(qs, thr, limit)
        for q, r in zip(qs, got):
            assert_exact(r, oi.score(q, thr, limit), f"g={g} q={q!r} thr={thr} limit={limit}")
    for q in qs[:16]:  # single-query API == batch API
        assert_exact(gi.score(q, 0.3, 20), oi.score(q, 0.3, 20), f"single g={g} q={q!r}")
        assert gi.search(q, 0.3, 20) == [k for k, _ in oi.score(q, 0.3, 20)]
    gi.dispose()


@pytest.mark.parametrize("g", [1, 2])
def test_narrow_gram_size_parity(g):
    rng = random.Random(40 + g)
    words, wts, _ = ssl.synth.gen_corpus(4000, seed=g, min_len=1, span=20, row_size=2)
    gi = ssl.StringIndex(words, 2, wts, gram_size=g)
    oi = OracleIndexG(words, 2, wts, g=g)
    assert gi.size() == oi.size() and gi.lib_size() == oi.lib_size()
    keys = [w for w in words[::2] if w]
    qs = []
    for i in range(64):
        src = rng.choice(keys)
        l = rng.randint(1, min(len(src), 3 * g + 6))
        o = rng.randrange(len(src) - l + 1)
        q = bytearray(src[o:o + l])
        if i % 3 == 0:
            q[rng.randrange(l)] = rng.choice(b"ABCXYZ")
        qs.append(bytes(q) if i % 4 else bytes(q).lower())
    qs += [b"", b"*", src, src + b" " + keys[0]]
    qs += [b"\xe9t\xe9 ABC", b"AB\xffCD"]
    for thr, limit in [(0.0, 100), (0.4, 10), (0.0, 0)]:
        for q, r in zip(qs, gi.score_batch(qs, thr, limit)):
            assert_exact(r, oi.score(q, thr, limit), f"g={g} q={q!r} thr={thr} limit={limit}")
    gi.dispose()


@pytest.mark.parametrize("g", [1, 2, 3])
def test_wide_tier2_limit_500_and_long_queries(g):
    """Tier 2 (k_fast) on dictionary-mode indexes: limits of 129..1024 and queries of 64..255
    grams are taken by k_fast (tier2_queries) instead of the library-wide general path, exact
    against the generic oracle; queries past 255 grams still go to the general path."""
    rng = random.Random(zlib.crc32(f"tier2w{g}".encode()))
    words, wts = _shape(wide_corpus(rng, 3000, 2, 6, 24), rng)
    gi = ssl.WideStringIndex(words, 2, wts, gram_size=g)
    gi.set_timing(True)  # per-call statistics (last_stats)
    oi = OracleIndexG(words, 2, wts, g=g, wide=True)
    keys = [w for w in words[::2] if w and w.strip()]
    qs = [q for q in wide_queries(rng, keys, 64) if isinstance(q, str) and len(q.strip()) > 3 * g + 2]
    for thr, limit in [(0.0, 500), (0.2, 1024), (0.4, 129)]:
        got = gi.score_batch(qs, thr, limit)
        st = gi.last_stats()
        assert st["tier2_queries"] > 0 and st["general_queries"] == 0, (thr, limit, st)
        for q, r in zip(qs, got):
            assert_exact(r, oi.score(q, thr, limit), f"tier2 g={g} q={q!r} thr={thr} limit={limit}")
    long_qs = []
    for i in range(12):
        src = rng.choice(keys)
        long_qs.append(((src + " ") * (300 // (len(src) + 1) + 1))[: 80 + 15 * i])  # 80..245 characters
    got = gi.score_batch(long_qs, 0.1, 100)
    st = gi.last_stats()
    assert st["tier2_queries"] == len(long_qs) and st["general_queries"] == 0, st
    for q, r in zip(long_qs, got):
        assert_exact(r, oi.score(q, 0.1, 100), f"tier2 long g={g} len={len(q)}")
    over = [(keys[0] + " ") * 40][:1]  # > 255 grams: the general path
    over = [over[0][: 256 + g + 4]]
    gi.score_batch(over, 0.1, 100)
    assert gi.last_stats()["general_queries"] == 1
    assert_exact(gi.score_batch(over, 0.1, 100)[0], oi.score(over[0], 0.1, 100), "tier2 over")
    gi.dispose()


@pytest.mark.parametrize("g", [1, 2])
def test_narrow_gram_size_tier2(g):
    """k_fast on narrow indexG libraries (dictionary of 1- or 2-byte grams) at limit 500."""
    rng = random.Random(70 + g)
    words, wts, _ = ssl.synth.gen_corpus(5000, seed=10 + g, min_len=4, span=20, row_size=1)
    gi = ssl.StringIndex(words, 1, wts, gram_size=g)
    gi.set_timing(True)
    oi = OracleIndexG(words, 1, wts, g=g)
    keys = [w for w in words if w]
    qs = [rng.choice(keys) for _ in range(40)] + [keys[1] + b" " + keys[2] for _ in range(4)]
    got = gi.score_batch(qs, 0.3, 500)
    st = gi.last_stats()
    assert st["tier2_queries"] == len(qs) and st["general_queries"] == 0, st
    for q, r in zip(qs, got):
        assert_exact(r, oi.score(q, 0.3, 500), f"narrow tier2 g={g} q={q!r}")
    gi.dispose()


def test_skewed_wide_lists_several_parts():
    # a 5-symbol alphabet of CJK characters: long lists split into several term-id parts
    rng = random.Random(77)
    words = wide_corpus(rng, 30000, 1, 6, 26, alpha="日本語中文")
    gi = ssl.WideStringIndex(words, 1, None, gram_size=2)
    oi = OracleIndexG(words, 1, None, g=2, wide=True)
    qs = wide_queries(rng, words, 40)
    for q, r in zip(qs, gi.score_batch(qs, 0.2, 50)):
        assert_exact(r, oi.score(q, 0.2, 50), f"skewed q={q!r}")


def test_wide_g3_ascii_equals_narrow_path():
    words, wts, rng = ssl.synth.gen_corpus(6000, seed=5, min_len=2, span=20)
    qs = ssl.synth.gen_queries(words, 1, 200, rng) + [b"", b"*", b"AB", b"abc de"]
    ni = ssl.StringIndex(words, 1, wts)
    wi = ssl.WideStringIndex([w.decode() for w in words], 1, wts, gram_size=3)
    assert ni.size() == wi.size() and ni.lib_size() == wi.lib_size()
    wres = wi.score_batch([q.decode() for q in qs], 0.25, 40)
    for q, n, w in zip(qs, ni.score_batch(qs, 0.25, 40), wres):
        assert_exact(w, [(k.decode(), s) for k, s in n], f"q={q!r}")


def test_width_mismatch_answers_zero():
    import ctypes as C
    from stringsearchlib_amd import _native
    L = _native.lib()
    ni = ssl.StringIndex([b"ALPHA BRAVO", b"CHARLIE DELTA"])
    wi = ssl.WideStringIndex(["ALPHA BRAVO", "CHARLIE DELTA"], gram_size=3)
    res = C.POINTER(C.POINTER(C.c_char))()
    assert L.search(wi.handle, b"ALPHA", C.byref(res), 0.0, 10) == 0 and not res
    wres = C.POINTER(C.POINTER(C.c_uint32))()
    q = (C.c_uint32 * 6)(*map(ord, "ALPHA"), 0)
    assert L.searchW(ni.handle, q, C.byref(wres), 0.0, 10) == 0 and not wres
    assert L.searchW(wi.handle, q, C.byref(wres), 0.0, 10) == 1
    L.releaseW(wi.handle, wres, None)
    assert L.ngsCharSize(ni.handle) == 1 and L.ngsCharSize(wi.handle) == 4
    assert not L.ngsKey(wi.handle, 0) and not L.ngsKeyW(ni.handle, 0)
    assert L.indexW(None, 0, 1, None, 0) == 0 and L.indexG(None, 0, 1, None, 4) == 0
    ni.dispose(); wi.dispose()


def test_wide_valid_char_changes():
    rng = random.Random(8)
    words = wide_corpus(rng, 2000, 1)
    gi = ssl.WideStringIndex(words, 1, None, gram_size=2)
    oi = OracleIndexG(words, 1, None, g=2, wide=True)
    qs = wide_queries(rng, words, 40)
    for valid in [b"ABCDEF ", bytes(range(1, 256))]:
        gi.set_valid_char(valid)
        oi.set_valid_char(valid)
        for q, r in zip(qs, gi.score_batch(qs, 0.2, 30)):
            assert_exact(r, oi.score(q, 0.2, 30), f"valid={valid[:6]!r} q={q!r}")


def test_wide_device_api_matches_host_api():
    torch = pytest.importorskip("torch")
    rng = random.Random(21)
    words = wide_corpus(rng, 5000, 1, 4, 20)
    qs = wide_queries(rng, words, 200)
    gi = ssl.WideStringIndex(words, 1, None, gram_size=2)
    units = [[ord(c) for c in q] if isinstance(q, str) else list(q) for q in qs]
    flat = b"".join(struct.pack(f"<{len(u)}I", *u) for u in units)
    offs = [0]
    for u in units:
        offs.append(offs[-1] + 4 * len(u))
    dev = torch.device("cuda:0")
    raw = torch.frombuffer(bytearray(flat) or bytearray(4), dtype=torch.uint8).to(dev)
    off = torch.tensor(offs, dtype=torch.int64, device=dev)
    limit = 50
    counts = torch.zeros(len(qs), dtype=torch.int32, device=dev)
    keys = torch.zeros(len(qs) * limit, dtype=torch.int32, device=dev)
    scores = torch.zeros(len(qs) * limit, dtype=torch.float32, device=dev)
    gi.search_device(raw.data_ptr(), off.data_ptr(), len(qs), 0.3, limit, limit, counts.data_ptr(),
                     keys.data_ptr(), scores.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c, k, s = counts.cpu().tolist(), keys.cpu().tolist(), scores.cpu().tolist()
    for i, h in enumerate(gi.score_batch(qs, 0.3, limit)):
        dv = [(gi.key(k[i * limit + j]), s[i * limit + j]) for j in range(c[i])]
        assert_exact(dv, h, f"device q={qs[i]!r}")
