"""Parity at BASELINE.json's full sizes (SURVEY.md §8(d) synthetic corpora).

C2 (1M rows, weight NULL, thr 0, limit 100, 4096 queries): every answer exact vs the oracle.
C3 (10M rows, weights, thr 0.3, limit 100, 65,536 queries): a seeded sample exact vs the
oracle; on every answer the size-independent properties (ordering, distinct keys, counts
within the limit, exact self-matches promoted to 100) and run-to-run determinism.
"""
import ctypes as C
import random
import struct

import pytest

from oracle_py import lib as olib
from tiecheck import bits

import scale_golden as sg

import stringsearchlib_amd as ssl
from stringsearchlib_amd import _native

pytestmark = pytest.mark.gpu


def corpus(rows):
    S = _native.synth()
    blob, wp, wt, st = C.c_void_p(), C.POINTER(C.c_char_p)(), C.POINTER(C.c_float)(), C.c_uint64()
    assert S.ngs_synth_corpus(rows, 42, 8, 17, 1, C.byref(blob), C.byref(wp), C.byref(wt), C.byref(st)) == 0
    return S, blob, wp, wt, st


def queries(S, wp, rows, st, n):
    state = C.c_uint64(st.value)
    qb, qo = C.c_void_p(), C.POINTER(C.c_uint64)()
    assert S.ngs_synth_queries(wp, rows, 1, n, C.byref(state), 12, C.byref(qb), C.byref(qo)) == 0
    raw = C.string_at(qb, qo[n])
    out = [raw[qo[i]:qo[i + 1]] for i in range(n)]
    S.ngs_synth_free(qb)
    S.ngs_synth_free(C.cast(qo, C.c_void_p))
    return out


def gpu_index(wp, wt, rows, weighted):
    L = _native.lib()
    h = L.indexN(wp, rows, 1, wt if weighted else None)
    assert h
    return h


def gpu_batch(h, qs, thr, limit):
    L = _native.lib()
    n = len(qs)
    arr = (C.c_char_p * n)(*qs)
    counts = (C.c_uint32 * n)()
    res = C.POINTER(C.POINTER(C.c_char))()
    sc = C.POINTER(C.c_float)()
    total = L.scoreBatch(h, arr, n, thr, limit, counts, C.byref(res), C.byref(sc))
    out, o = [], 0
    for i in range(n):
        out.append([(C.string_at(res[o + j]), sc[o + j]) for j in range(counts[i])])
        o += counts[i]
    assert o == total
    L.release(h, res, sc)
    return out


def oracle_batch(oh, qs, thr, limit):
    O = olib()
    n = len(qs)
    arr = (C.c_char_p * n)(*qs)
    counts = (C.c_uint32 * n)()
    keys = (C.c_uint32 * (n * limit))()
    scores = (C.c_float * (n * limit))()
    O.ngo_search_batch(oh, arr, n, thr, limit, counts, keys, scores, limit, 8)
    out = []
    for i in range(n):
        row = []
        for j in range(counts[i]):
            ln = C.c_uint32()
            p = O.ngo_key(oh, keys[i * limit + j], C.byref(ln))
            row.append((C.string_at(p, ln.value), scores[i * limit + j]))
        out.append(row)
    return out


def assert_same(a, b, where):
    assert len(a) == len(b), f"{where}: {len(a)} vs {len(b)}"
    for (k1, s1), (k2, s2) in zip(a, b):
        assert k1 == k2 and bits(s1) == bits(s2), f"{where}: {k1!r}|{s1} vs {k2!r}|{s2}"


def check_small_batches(h, qs, got, thr, limit, idx, where):
    """The latency path (batches of <= 16 queries: a wave per (query, term-id slice) and k_merge on
    a large library) gives the batch path's answers."""
    for i0 in range(0, len(idx), 16):
        part = idx[i0:i0 + 16]
        for i, g in zip(part, gpu_batch(h, [qs[i] for i in part], thr, limit)):
            assert_same(g, got[i], f"{where} small batch q#{i}")
    for i in idx[:24]:
        assert_same(gpu_batch(h, [qs[i]], thr, limit)[0], got[i], f"{where} single q#{i}")


def check_properties(res, limit, where):
    assert len(res) <= limit, where
    keys = [k for k, _ in res]
    assert len(set(keys)) == len(keys), f"{where}: duplicate key"
    for (k1, s1), (k2, s2) in zip(res, res[1:]):
        assert s1 > s2 or (s1 == s2 and len(k1) <= len(k2)), f"{where}: order {k1!r}|{s1} {k2!r}|{s2}"


def test_c2_full_exact():
    rows, B = 1_000_000, 4096
    S, blob, wp, wt, st = corpus(rows)
    h = gpu_index(wp, wt, rows, False)
    oh = olib().ngo_build(wp, rows, 1, None)
    qs = queries(S, wp, rows, st, B)
    got = gpu_batch(h, qs, 0.0, 100)
    ref = oracle_batch(oh, qs, 0.0, 100)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert_same(g, r, f"C2 q#{i} {qs[i]!r}")
    check_small_batches(h, qs, got, 0.0, 100, list(range(96)), "C2")
    olib().ngo_free(oh)
    _native.lib().dispose(h)


def test_c3_full_sampled_exact_and_properties():
    rows, B = 10_000_000, 65536
    S, blob, wp, wt, st = corpus(rows)
    h = gpu_index(wp, wt, rows, True)
    qs = queries(S, wp, rows, st, B)
    rng = random.Random(7)
    exact_rows = [rng.randrange(rows) for _ in range(64)]
    qs += [wp[i] for i in exact_rows]  # a row's own key: promoted to 100
    got = gpu_batch(h, qs, 0.3, 100)
    for i, g in enumerate(got):
        check_properties(g, 100, f"C3 q#{i}")
    for j, r in enumerate(exact_rows):
        assert got[B + j][0] == (wp[r], 100.0)
    again = gpu_batch(h, qs[:4096], 0.3, 100)
    for i in range(4096):
        assert_same(again[i], got[i], f"C3 rerun q#{i}")
    check_small_batches(h, qs, got, 0.3, 100, list(range(B, B + 8)) + list(range(88)), "C3")
    oh = olib().ngo_build(wp, rows, 1, wt)
    sample = sorted(rng.sample(range(len(qs)), 4096))
    ref = oracle_batch(oh, [qs[i] for i in sample], 0.3, 100)
    for i, r in zip(sample, ref):
        assert_same(got[i], r, f"C3 q#{i} {qs[i]!r}")
    olib().ngo_free(oh)
    _native.lib().dispose(h)


@pytest.mark.parametrize("name", sg.available())
def test_reference_answers_at_scale(name):
    """The HIP path against the REFERENCE DLL's own answers at C2 / C3 scale (tie-aware;
    tests/golden/scale, written by tests/golden/make_golden_scale.py)."""
    fx = sg.load(name)
    spec = fx["spec"]
    S, blob, wp, wt, st = sg.corpus(spec)
    h = _native.lib().indexN(wp, spec["rows"] * spec["row_size"], spec["row_size"], wt if spec["weights"] else None)
    assert h
    L = _native.lib()
    assert L.getSize(h) == fx["size"] and L.getLibSize(h) == fx["libSize"]
    qs = sg.queries(fx)
    sg.check_answers(fx, gpu_batch(h, qs, spec["thr"], spec["limit"]), "GPU batch")
    # the latency path (batches of <= 16, 32 term-id slices per query) on the same queries
    for i0 in range(0, 64, 16):
        sg.check_answers({"name": fx["name"], "cases": fx["cases"][i0:i0 + 16]},
                         gpu_batch(h, qs[i0:i0 + 16], spec["thr"], spec["limit"]), "GPU small batch")
    L.dispose(h)
    sg.free(S, blob, wp, wt)
