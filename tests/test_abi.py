"""CPU-side checks of the drop-in boundary (no GPU compute)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from stringsearchlib_amd import _native

REF_EXPORTS = ["indexN", "search", "score", "release", "dispose", "getSize", "getLibSize", "setValidChar"]


def test_header_declares_reference_exports():
    syms = _native.declared_symbols()
    for s in REF_EXPORTS:  # nGramSearch/dllmain.cpp:37-151
        assert s in syms
    # README-only `index` must not be exported (it collides with glibc's index(3)), SURVEY §7
    assert "index" not in syms


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (\w+)$", out, re.M))
    missing = [s for s in _native.declared_symbols() if s not in exported]
    assert not missing, missing


def test_library_loads_and_binds():
    L = _native.lib()
    for s in _native.declared_symbols():
        assert hasattr(L, s)
    assert b"gfx950" in L.ngsVersion()


def test_reference_signatures_match_header():
    """The eight reference prototypes are reproduced verbatim (modulo const on pointers
    the reference declares `char** const` / `float* const`, which is not part of the ABI)."""
    text = open(_native.HEADER).read()
    want = {
        "indexN": r"uint32_t indexN\(char\*\* words, uint64_t size, uint16_t rowSize, float\* weight\)",
        "search": r"uint32_t search\(uint32_t handle, const char\* query, char\*\*\* results, float threshold,\s+uint32_t limit\)",
        "score": r"uint32_t score\(uint32_t handle, const char\* query, char\*\*\* results, float\*\* scores,\s+float threshold, uint32_t limit\)",
        "release": r"void release\(uint32_t handle, char\*\* results, float\* scores\)",
        "dispose": r"void dispose\(uint32_t handle\)",
        "getSize": r"uint64_t getSize\(uint32_t handle\)",
        "getLibSize": r"uint64_t getLibSize\(uint32_t handle\)",
        "setValidChar": r"void setValidChar\(uint32_t handle, char\* characters, int n\)",
    }
    for name, pat in want.items():
        assert re.search(pat, text), name


def test_unbuilt_library_without_gpu_work():
    """size < 2 gives a handle whose searches return 0 and leave outputs untouched
    (nGramSearch.hpp:122-123, dllmain.cpp:61-69) — no device work is involved."""
    L = _native.lib()
    words = (C.c_char_p * 1)(b"ONLY")
    h = L.indexN(words, 1, 1, None)
    assert h
    try:
        assert L.getSize(h) == 0 and L.getLibSize(h) == 0
        sentinel = C.POINTER(C.POINTER(C.c_char))()
        assert L.search(h, b"ONLY", C.byref(sentinel), 0.0, 10) == 0
        assert not sentinel
        assert L.search(h + 1000, b"x", C.byref(sentinel), 0.0, 10) == 0  # unknown handle
    finally:
        L.dispose(h)
    assert L.getSize(h) == 0


def test_wide_and_gram_size_entry_points_without_gpu_work():
    """indexG / indexW validate gSize (1..3) and, like indexN, give an un-built handle for a
    library of < 2 words; width-mismatched or un-built searches answer 0."""
    L = _native.lib()
    words = (C.c_char_p * 1)(b"ONLY")
    assert L.indexG(words, 1, 1, None, 0) == 0 and L.indexG(words, 1, 1, None, 4) == 0
    U = C.POINTER(C.c_uint32)
    w0 = (C.c_uint32 * 5)(*map(ord, "ONLY"), 0)
    wwords = (U * 1)(C.cast(w0, U))
    assert L.indexW(wwords, 1, 1, None, 0) == 0
    h = L.indexW(wwords, 1, 1, None, 2)
    assert h
    try:
        assert L.ngsCharSize(h) == 4 and L.ngsGramSize(h) == 2
        assert L.getSizeW(h) == 0 and L.getLibSizeW(h) == 0
        res = C.POINTER(U)()
        assert L.searchW(h, C.cast(w0, U), C.byref(res), 0.0, 10) == 0 and not res
        nres = C.POINTER(C.POINTER(C.c_char))()
        assert L.search(h, b"ONLY", C.byref(nres), 0.0, 10) == 0 and not nres
    finally:
        L.disposeW(h)
    assert L.ngsCharSize(h) == 0
