"""The CPU restatement (oracle/ngs_oracle.c) against the REFERENCE at the benchmark's scale:
BASELINE configs[1] (C2, 1M rows, threshold 0) and configs[2] (C3, 10M rows, weights, threshold
0.3), tie-aware against the reference DLL's own answers (tests/golden/scale, see
tests/golden/make_golden_scale.py). This pins the oracle that the GPU tests compare with
exactly at the sizes where the GPU runs, not only on the small fixtures."""
import ctypes as C

import pytest

import scale_golden as sg
from oracle_py import lib as olib


@pytest.mark.parametrize("name", sg.available())
@pytest.mark.timeout(600)
def test_oracle_matches_reference_at_scale(name):
    fx = sg.load(name)
    spec = fx["spec"]
    S, blob, wp, wt, st = sg.corpus(spec)
    O = olib()
    n_words = spec["rows"] * spec["row_size"]
    oh = O.ngo_build(wp, n_words, spec["row_size"], wt if spec["weights"] else None)
    assert O.ngo_size(oh) == fx["size"] and O.ngo_libsize(oh) == fx["libSize"]
    qs = sg.queries(fx)
    n, limit = len(qs), spec["limit"]
    arr = (C.c_char_p * n)(*qs)
    counts = (C.c_uint32 * n)()
    keys = (C.c_uint32 * (n * limit))()
    scores = (C.c_float * (n * limit))()
    O.ngo_search_batch(oh, arr, n, spec["thr"], limit, counts, keys, scores, limit, 8)
    answers = []
    for i in range(n):
        row = []
        for j in range(counts[i]):
            ln = C.c_uint32()
            p = O.ngo_key(oh, keys[i * limit + j], C.byref(ln))
            row.append((C.string_at(p, ln.value), scores[i * limit + j]))
        answers.append(row)
    sg.check_answers(fx, answers, "oracle")
    O.ngo_free(oh)
    sg.free(S, blob, wp, wt)
