"""BASELINE.json configs[3] and configs[4] at their full shapes (the bench's synthetic corpora).

C4: 10M rows of UTF-32 strings through indexW with gSize 2 and rowSize 4 (a key and 3 aliases:
40M words), 2-grams over a 37-symbol alphabet, so the posting lists are dense (~440k postings)
and the skip table takes 32,768 buckets. Checked on the full 65,536-query batch, three times (the
first call grows the survivor arena): every count within the limit, properties on 4,096 decoded
answers, a seeded sample exact against oracle/ngs_oracle_g.c (the gram-size / UTF-32
restatement; parity unpinned beyond g = 3, see test_oracle_generic.py), the batch answer equal
to per-query answers, and the context's survivor memory within 2 GiB: queries whose survivors
outgrow their 2,048 slots (the wide cap at 65,536 queries) go on in the batch-wide arena instead
of growing every query's slots (round 4: 32,768 slots per query, 10 GiB).

C5: the per-GPU slice of the 8-GPU config: a 50M-row library (weight NULL) and 131,072 queries
(2^20 / 8). Checked: properties on every answer, exact self-matches promoted to 100, a seeded
sample exact against oracle/ngs_oracle.c (pinned to the reference), run-to-run determinism.
"""
import ctypes as C
import random

import pytest

import bench
from oracle_py import lib as olib, lib_g
from test_gpu_fullsize import assert_same, check_properties, gpu_batch, oracle_batch, queries, corpus

from stringsearchlib_amd import _native

pytestmark = pytest.mark.gpu

U32P = C.POINTER(C.c_uint32)


def _wide_arr(qs):
    bufs = [(C.c_uint32 * (len(q) + 1))(*q, 0) for q in qs]
    return bufs, (U32P * len(qs))(*[C.cast(b, U32P) for b in bufs])


def _wstr(p):
    out, i = [], 0
    while p[i]:
        out.append(p[i])
        i += 1
    return tuple(out)


def gpu_batch_w(h, qs, thr, limit, decode=None):
    """scoreBatchW; the answers of the queries in `decode` (all if None) as lists, the others None,
    and the counts."""
    L = _native.lib()
    n = len(qs)
    bufs, arr = _wide_arr(qs)
    counts = (C.c_uint32 * n)()
    res = C.POINTER(U32P)()
    sc = C.POINTER(C.c_float)()
    total = L.scoreBatchW(h, arr, n, thr, limit, counts, C.byref(res), C.byref(sc))
    want = None if decode is None else set(decode)
    out, o = [], 0
    for i in range(n):
        out.append([(_wstr(res[o + j]), sc[o + j]) for j in range(counts[i])] if want is None or i in want else None)
        o += counts[i]
    assert o == total
    L.releaseW(h, res, sc)
    return out if decode is None else (out, list(counts))


def oracle_batch_w(oh, qs, thr, limit, threads=16):
    O = lib_g()
    n = len(qs)
    bufs, arr = _wide_arr(qs)
    counts = (C.c_uint32 * n)()
    keys = (C.c_uint32 * (n * limit))()
    scores = (C.c_float * (n * limit))()
    O.ngog_search_batch(oh, arr, n, thr, limit, counts, keys, scores, limit, threads)
    out = []
    for i in range(n):
        row = []
        for j in range(counts[i]):
            ln = C.c_uint32()
            p = O.ngog_key(oh, keys[i * limit + j], C.byref(ln))
            row.append((tuple(p[k] for k in range(ln.value)), scores[i * limit + j]))
        out.append(row)
    return out


def test_c4_full_wide_g2_rowsize4():
    cfg = bench.CONFIGS["c4"]
    corpus4 = bench.Corpus(cfg["rows"], row_size=cfg["row_size"], wide=True)
    h = bench.build_index(corpus4, False, 0, gram=cfg["gram"])
    L = _native.lib()
    assert L.ngsCharSize(h) == 4 and L.ngsGramSize(h) == 2 and L.getSize(h) > 0
    raw, offs = corpus4.queries(cfg["batch"])
    qs = [tuple(raw[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]  # ASCII: one byte per code point
    rng = random.Random(4)
    sample = sorted(rng.sample(range(len(qs)), 40))
    decode = sorted(set(rng.sample(range(len(qs)), 4096)) | set(sample))
    L.ngsSetTiming(h, 1)
    st = _native.NgsStats()
    for call in range(3):
        got, counts = gpu_batch_w(h, qs, cfg["threshold"], cfg["limit"], decode=decode)
        L.ngsLastStats(h, C.byref(st))
        assert max(counts) <= cfg["limit"] and sum(counts) > 0
        # survivors past the query's slots went on in the arena; no query's slots grew
        assert st.survivor_slots == 2048 and st.survivor_slot_bytes <= 2 << 30, (st.survivor_slots, st.survivor_slot_bytes)
        if call == 2:  # the arena held every overflow: no query handed over for its slots
            assert st.arena_used <= st.arena_blocks and st.slot_full_queries == 0, (st.arena_used, st.arena_blocks)
    assert st.arena_used > 0  # C4's long tail of survivors (3,962 per query on average) needs it
    for i in decode:
        check_properties(got[i], cfg["limit"], f"C4 q#{i}")
    for i in sample[:8]:  # the batch answer is each query's own answer
        assert gpu_batch_w(h, [qs[i]], cfg["threshold"], cfg["limit"])[0] == got[i]
    oh = lib_g().ngog_build(corpus4.wwords, corpus4.n_words, corpus4.row_size, None, cfg["gram"], 1)
    ref = oracle_batch_w(oh, [qs[i] for i in sample], cfg["threshold"], cfg["limit"])
    for i, r in zip(sample, ref):
        assert_same(got[i], r, f"C4 q#{i} {bytes(qs[i])!r}")
    # limit 500: tier 2 (k_fast) on the dictionary-mode index, not the library-wide general path
    wide500 = [qs[i] for i in sample[:24]]
    L.ngsSetTiming(h, 1)
    got500 = gpu_batch_w(h, wide500, cfg["threshold"], 500)
    st = _native.NgsStats()
    L.ngsLastStats(h, C.byref(st))
    assert st.tier2_queries > 0 and st.general_queries == 0, (st.tier2_queries, st.general_queries)
    ref500 = oracle_batch_w(oh, wide500, cfg["threshold"], 500)
    for j, (g500, r) in enumerate(zip(got500, ref500)):
        check_properties(g500, 500, f"C4 limit 500 q#{j}")
        assert_same(g500, r, f"C4 limit 500 q#{j}")
    lib_g().ngog_free(oh)
    L.dispose(h)
    corpus4.free()


def test_c5_slice_full_sampled_exact_and_properties():
    cfg = bench.CONFIGS["c5"]
    rows, B = cfg["rows"], cfg["batch"]
    S, blob, wp, wt, st = corpus(rows)
    L = _native.lib()
    h = L.indexN(wp, rows, 1, None)
    assert h and L.getSize(h) > 0
    qs = queries(S, wp, rows, st, B)
    rng = random.Random(5)
    exact_rows = [rng.randrange(rows) for _ in range(64)]
    qs += [wp[i] for i in exact_rows]  # a row's own key: promoted to 100
    got = gpu_batch(h, qs, cfg["threshold"], cfg["limit"])
    for i, g in enumerate(got):
        check_properties(g, cfg["limit"], f"C5 q#{i}")
    for j, r in enumerate(exact_rows):
        assert got[B + j][0] == (wp[r], 100.0)
    again = gpu_batch(h, qs[:4096], cfg["threshold"], cfg["limit"])
    for i in range(4096):
        assert_same(again[i], got[i], f"C5 rerun q#{i}")
    oh = olib().ngo_build(wp, rows, 1, None)
    sample = sorted(rng.sample(range(len(qs)), 384))
    ref = oracle_batch(oh, [qs[i] for i in sample], cfg["threshold"], cfg["limit"])
    for i, r in zip(sample, ref):
        assert_same(got[i], r, f"C5 q#{i} {qs[i]!r}")
    olib().ngo_free(oh)
    L.dispose(h)
    for p in (blob, C.cast(wp, C.c_void_p), C.cast(wt, C.c_void_p)):
        S.ngs_synth_free(p)
