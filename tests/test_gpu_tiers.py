"""Every kernel tier of the search path, driven on purpose and checked exactly against the oracle.

Routing (ngs_kernels.hip: heavy_class, wave_query's hand-over, fast_one's guard):
* tier 1a (k_wave_lean + k_emit): <= 63 grams, limit <= 128, cmin >= 3, no short search;
* heavy list (k_wave_lean on a side stream): cmin 2 (8-character queries at thr 0.3);
* full list / hand-overs (k_wave, tier 1b): cmin 1 (thr 0) or a short search (|q| < 9);
* tier 2 (k_fast, one block per query): 64..255 grams (66..257 bytes) or limit 129..1024;
* general (k_gen_*): |q| <= 3 (full-library scan), > 255 grams, or limit > 1024.

Each test asserts the path counts of ngsLastStats so a routing change cannot silently bypass
the tier it is meant to cover. The reference behaviour is nGramSearch.hpp:278-301 (searchLong),
:310-341 (calcScore) and :397-401 (partial_sort to limit).
"""
import random
import zlib

import pytest

from oracle_py import OracleIndex
from test_gpu_parity import _corpus, assert_exact

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu


def _check(gi, oi, qs, thr, limit, where):
    gi.set_timing(True)
    got = gi.score_batch(qs, thr, limit)
    st = gi.last_stats()
    for q, g in zip(qs, got):
        assert_exact(g, oi.score(q, thr, limit), f"{where} q={q[:40]!r}.. len={len(q)} thr={thr} limit={limit}")
    return st


def _long_queries(rng, words, n, lo=66, hi=257):
    """Queries of lo..hi normalised bytes: keys glued with spaces, cut, one substitution."""
    keys = [w for w in words if w]
    out = []
    for i in range(n):
        target = lo + (i * 37) % (hi - lo + 1) if i > 1 else (lo if i == 0 else hi)
        parts, size = [], 0
        while size < target:
            k = rng.choice(keys)
            parts.append(k)
            size += len(k) + 1
        q = bytearray(b" ".join(parts)[:target].strip())
        while len(q) < target:  # a trailing space was trimmed: pad with a letter
            q += b"Q"
        if i % 3 == 1:
            q[rng.randrange(len(q))] = ord(rng.choice("ABCDEFGHIJKLMNOPQRSTUVWXYZ"))
        out.append(bytes(q))
    return out


def _short_windows(rng, words, n, qlen=12):
    keys = [w for w in words if w and len(w) >= qlen] or [w for w in words if w and len(w) >= 4]
    out = []
    for _ in range(n):
        src = rng.choice(keys)
        l = min(qlen, len(src))
        o = rng.randrange(len(src) - l + 1)
        q = bytearray(src[o:o + l])
        q[rng.randrange(l)] = ord(rng.choice("ABCDEFGHIJKLMNOPQRSTUVWXYZ"))
        out.append(bytes(q))
    return out


@pytest.fixture(scope="module")
def bench20k():
    words, wts, _ = ssl.synth.gen_corpus(20000, seed=21)
    gi, oi = ssl.StringIndex(words, 1, wts), OracleIndex(words, 1, wts)
    yield words, gi, oi
    gi.dispose()


@pytest.mark.parametrize("thr", [0.0, 0.3, 1.0])
def test_tier2_by_gram_count(bench20k, thr):
    """66..257-byte queries (64..255 grams) go to k_fast and finish there."""
    words, gi, oi = bench20k
    rng = random.Random(int(thr * 10) + 1)
    qs = _long_queries(rng, words, 40)
    assert min(map(len, qs)) == 66 and max(map(len, qs)) == 257
    st = _check(gi, oi, qs, thr, 100, "tier2-grams")
    assert st["tier2_queries"] == len(qs), st
    assert st["general_queries"] == 0, st  # every one finished inside tier 2
    assert st["fast_queries"] == len(qs), st


def test_tier2_gram_count_edges(bench20k):
    """65 bytes (63 grams) stays in tier 1; 66 and 257 go to tier 2 and finish there; 258 is
    listed for tier 2 by tier 1 (> 63 grams) and passed on by k_fast to the general path."""
    words, gi, oi = bench20k
    rng = random.Random(7)
    for length, tier2, general in [(65, 0, 0), (66, 1, 0), (257, 1, 0), (258, 1, 1)]:
        qs = _long_queries(rng, words, 3, lo=length, hi=length)
        assert all(len(q) == length for q in qs)
        st = _check(gi, oi, qs, 0.3, 100, f"edge-{length}")
        assert st["tier2_queries"] == tier2 * len(qs), (length, st)
        assert st["general_queries"] == general * len(qs), (length, st)
        assert st["fast_queries"] == (1 - general) * len(qs), (length, st)


@pytest.mark.parametrize("limit", [129, 500, 1024])
@pytest.mark.parametrize("thr", [0.0, 0.3])
def test_tier2_by_limit(bench20k, thr, limit):
    """Limits 129..1024 route 12-byte queries to k_fast; a limit of 1025 goes general."""
    words, gi, oi = bench20k
    rng = random.Random(limit + int(thr * 10))
    qs = _short_windows(rng, words, 32) + _long_queries(rng, words, 4)
    st = _check(gi, oi, qs, thr, limit, "tier2-limit")
    assert st["tier2_queries"] == len(qs), st
    assert st["general_queries"] == 0, st


@pytest.mark.parametrize("kind", ["skewed", "rows", "short"])
@pytest.mark.parametrize("thr,limit", [(0.0, 300), (0.3, 1024), (1.0, 129), (0.3, 100)])
def test_tier2_other_corpora(kind, thr, limit):
    """Skewed lists (bucket sub-parts in tier 2's planner), aliases / NULL holes / zero and
    negative weights, and short terms (tier 2's register Levenshtein over shortLib)."""
    rng = random.Random(zlib.crc32(kind.encode()))
    words, rs, wts = _corpus(kind, random.Random(11))
    gi, oi = ssl.StringIndex(words, rs, wts), OracleIndex(words, rs, wts)
    live = [w for w in words if w]
    qs = _short_windows(rng, live, 16) + _long_queries(rng, live, 8, 66, 140)
    if kind == "short":
        qs += [w[:rng.randint(4, 8)] for w in rng.sample([w for w in live if len(w) >= 4], 8)]
    st = _check(gi, oi, qs, thr, limit, f"{kind}")
    assert st["fast_queries"] + st["general_queries"] == len(qs), st
    if limit > 128:
        assert st["tier2_queries"] == len(qs) and st["general_queries"] == 0, st
    else:
        assert st["tier2_queries"] >= 8, st  # the long queries
    gi.dispose()


def test_tier1a_only(bench20k):
    """C3-shaped queries (12 bytes, thr 0.3: cmin 3) finish in the lean kernel: no heavy, full,
    hand-over, tier-2 or general query."""
    words, gi, oi = bench20k
    qs = _short_windows(random.Random(3), words, 64)
    st = _check(gi, oi, qs, 0.3, 100, "tier1a")
    assert st["fast_queries"] == len(qs), st
    for k in ("heavy_queries", "full_queries", "handover_queries", "tier2_queries", "general_queries"):
        assert st[k] == 0, (k, st)


def test_heavy_and_full_lists(bench20k):
    """8-character queries at thr 0.3 (cmin 2) and 12-character ones at thr 0 (cmin 1, part_ones)
    take the heavy list into the lean kernel."""
    words, gi, oi = bench20k
    rng = random.Random(4)
    q8 = _short_windows(rng, words, 32, qlen=8)
    st = _check(gi, oi, q8, 0.3, 100, "heavy")
    assert st["heavy_queries"] == len(q8) and st["full_queries"] == 0, st
    q12 = _short_windows(rng, words, 32)
    st = _check(gi, oi, q12, 0.0, 100, "ones")
    assert st["heavy_queries"] == len(q12) and st["full_queries"] == 0, st
    assert st["handover_queries"] < len(q12) // 4, st  # most finish in part_ones
    # (this corpus has no shortLib, keys of 8-24 characters: the full list's short-search case
    # is routed in test_gpu_heavy.py)
    _check(gi, oi, _short_windows(rng, words, 32, qlen=7), 0.0, 100, "ones-7")


def test_general_path(bench20k):
    """|q| <= 3 scans the whole library; > 255 grams and limit > 1024 go general too."""
    words, gi, oi = bench20k
    rng = random.Random(5)
    qs = [w[:rng.randint(1, 3)] for w in rng.sample(words, 6)]
    st = _check(gi, oi, qs, 0.0, 100, "general-short")
    assert st["general_queries"] == len(qs), st
    qs = _short_windows(rng, words, 6)
    st = _check(gi, oi, qs, 0.3, 1500, "general-limit")
    assert st["general_queries"] == len(qs), st


def test_device_api_general_path_without_device_sync(bench20k):
    """ngsSearchDevice on torch's current stream: general-path answers (|q| <= 3, limit 0) are
    complete when the call returns, read back with no device-wide synchronisation."""
    import torch
    words, gi, oi = bench20k
    qs = [b"AB", b"A", words[5], b"XYZ", words[9][:3]]
    dev = torch.device("cuda", 0)
    raw = b"".join(qs)
    offs = [0]
    for q in qs:
        offs.append(offs[-1] + len(q))
    d_raw = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    stride = gi.num_keys()
    for rep in range(2):
        d_cnt = torch.full((len(qs),), 7, dtype=torch.int32, device=dev)
        d_key = torch.full((len(qs) * stride,), -1, dtype=torch.int32, device=dev)
        d_sc = torch.zeros(len(qs) * stride, dtype=torch.float32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        gi.search_device(d_raw.data_ptr(), d_off.data_ptr(), len(qs), 0.0, 0, stride, d_cnt.data_ptr(),
                         d_key.data_ptr(), d_sc.data_ptr(), stream)
        cnt, key, sc = d_cnt.cpu().tolist(), d_key.cpu().tolist(), d_sc.cpu().tolist()
        for i, q in enumerate(qs):
            ref = oi.score(q, 0.0, 0)
            got = [(gi.key(key[i * stride + j]), sc[i * stride + j]) for j in range(cnt[i])]
            assert_exact(got, ref, f"device q={q!r} rep={rep}")


@pytest.mark.parametrize("kind", ["bench", "rows", "short"])
def test_general_select_limits(bench20k, kind):
    """The general path's top-L (k_gen_select: radix select over the row of key encodings, the
    first keys at the L-th score in key order, an LDS sort) at limits that cut through long runs
    of equal scores, limits above the number of scored keys, and 1025 (the per-query sort) —
    exact against the oracle, with more queries than one group holds."""
    if kind == "bench":
        words, gi, oi = bench20k
        own = False
    else:
        words, rs, wts = _corpus(kind, random.Random(13))
        gi, oi = ssl.StringIndex(words, rs, wts), OracleIndex(words, rs, wts)
        own = True
    rng = random.Random(zlib.crc32(kind.encode()) + 1)
    live = [w for w in words if w]
    base = [w[:rng.randint(1, 3)] for w in rng.sample(live, 24)] + [b"E", b"ZZ", b"Q9X"]
    for thr, limit in [(0.0, 1), (0.0, 2), (0.3, 37), (0.5, 100), (0.0, 1024), (1.0, 1024), (0.3, 1025)]:
        st = _check(gi, oi, base, thr, limit, f"general-select-{kind}")
        assert st["general_queries"] == len(base), st
    many = [w[:rng.randint(2, 3)] for w in rng.sample(live, 150)]
    st = _check(gi, oi, many, 0.3, 100, f"general-groups-{kind}")
    assert st["general_queries"] == len(many), st
    if own:
        gi.dispose()
