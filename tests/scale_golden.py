"""The reference's answers at the benchmark's scale (tests/golden/scale/*.json, written by
tests/golden/make_golden_scale.py from the reference DLL itself) and the check against them.

A fixture holds the generator spec of its corpus (csrc/synth.c, seed 42), the
queries (the first 256 of the bench's query stream, plus rows' own keys at C3) and, per query,
the reference's result count at the limit and its full ranking cut after the boundary
(score, key length) class. Answers are compared tie-aware (tests/tiecheck.py).
"""
from __future__ import annotations

import ctypes as C
import json
import os

from tiecheck import check

HERE = os.path.dirname(os.path.abspath(__file__))
SCALE = os.path.join(HERE, "golden", "scale")


def load(name: str) -> dict:
    with open(os.path.join(SCALE, f"{name}.json")) as f:
        return json.load(f)


def available() -> list[str]:
    return sorted(p[:-5] for p in os.listdir(SCALE) if p.endswith(".json")) if os.path.isdir(SCALE) else []


def corpus(spec):
    """(synth lib, blob, words, weights, state) of the fixture's corpus, from csrc/synth.c."""
    from stringsearchlib_amd import _native
    S = _native.synth()
    blob, wp, wt, st = C.c_void_p(), C.POINTER(C.c_char_p)(), C.POINTER(C.c_float)(), C.c_uint64()
    assert S.ngs_synth_corpus(spec["rows"], spec["seed"], spec["min_len"], spec["span"], spec["row_size"],
                              C.byref(blob), C.byref(wp), C.byref(wt), C.byref(st)) == 0
    return S, blob, wp, wt, st


def free(S, blob, wp, wt):
    for p in (blob, C.cast(wp, C.c_void_p), C.cast(wt, C.c_void_p)):
        S.ngs_synth_free(p)


def queries(fx) -> list[bytes]:
    return [c["q"].encode("latin-1") for c in fx["cases"]]


def check_answers(fx, answers, who: str) -> None:
    """answers[i]: list of (key bytes, fp32 score) for fixture query i."""
    assert len(answers) == len(fx["cases"])
    for i, (c, ours) in enumerate(zip(fx["cases"], answers)):
        check(ours, c["n"], [k.encode("latin-1") for k in c["full_keys"]], c["full_scores"],
              f"{fx['name']} {who} q#{i} {c['q']!r}")
