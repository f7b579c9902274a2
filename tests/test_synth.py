"""The C synthetic generator (bench) is byte-identical to the Python statement."""
import ctypes as C

from stringsearchlib_amd import _native
from stringsearchlib_amd.synth import SplitMix64, gen_corpus, gen_queries


def test_c_and_python_generators_agree():
    S = _native.synth()
    for rows, min_len, span, rs in [(500, 8, 17, 1), (300, 1, 12, 4)]:
        words, weights, rng = gen_corpus(rows, seed=42, min_len=min_len, span=span, row_size=rs)
        state_after_rows = rng.s
        qs = gen_queries(words, rs, 200, rng)
        blob, wp, wt, st = C.c_void_p(), C.POINTER(C.c_char_p)(), C.POINTER(C.c_float)(), C.c_uint64()
        assert S.ngs_synth_corpus(rows, 42, min_len, span, rs, C.byref(blob), C.byref(wp), C.byref(wt),
                                  C.byref(st)) == 0
        assert [wp[i] for i in range(rows * rs)] == words
        assert [wt[i] for i in range(rows * rs)] == weights
        assert st.value == state_after_rows
        qb, qo = C.c_void_p(), C.POINTER(C.c_uint64)()
        state = C.c_uint64(st.value)
        assert S.ngs_synth_queries(wp, rows * rs, rs, 200, C.byref(state), 12, C.byref(qb), C.byref(qo)) == 0
        raw = C.string_at(qb, qo[200])
        assert [raw[qo[i]:qo[i + 1]] for i in range(200)] == qs
        for p in (blob, C.cast(wp, C.c_void_p), C.cast(wt, C.c_void_p), qb, C.cast(qo, C.c_void_p)):
            S.ngs_synth_free(p)


def test_splitmix_known_values():
    r = SplitMix64(0)
    assert r.next() == 0xE220A8397B1DCDAF  # splitmix64 reference output for seed 0
