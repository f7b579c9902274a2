"""ctypes binding of the CPU restatement (libngs_oracle.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libngs_oracle.so")
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.ngo_build.restype = C.c_void_p
        L.ngo_build.argtypes = [C.POINTER(C.c_char_p), C.c_uint64, C.c_uint16, C.POINTER(C.c_float)]
        L.ngo_free.argtypes = [C.c_void_p]
        L.ngo_indexed.argtypes = [C.c_void_p]
        L.ngo_size.restype = C.c_uint64
        L.ngo_size.argtypes = [C.c_void_p]
        L.ngo_libsize.restype = C.c_uint64
        L.ngo_libsize.argtypes = [C.c_void_p]
        L.ngo_nkeys.restype = C.c_uint32
        L.ngo_nkeys.argtypes = [C.c_void_p]
        L.ngo_key.restype = C.POINTER(C.c_char)
        L.ngo_key.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.ngo_set_valid.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
        L.ngo_search.restype = C.c_uint32
        L.ngo_search.argtypes = [C.c_void_p, C.c_char_p, C.c_float, C.c_uint32, C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_float), C.c_uint32]
        L.ngo_search_amb.restype = C.c_uint32
        L.ngo_search_amb.argtypes = [C.c_void_p, C.c_char_p, C.c_float, C.c_uint32, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_float), C.c_uint32, C.POINTER(C.c_int)]
        L.ngo_search_batch.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.c_uint32, C.c_float, C.c_uint32,
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_float),
                                       C.c_uint32, C.c_int]
        _lib = L
    return _lib


def _words_array(words):
    arr = (C.c_char_p * max(1, len(words)))()
    for i, w in enumerate(words):
        arr[i] = None if w is None else (w if isinstance(w, bytes) else w.encode("latin-1"))
    return arr


class OracleIndex:
    """CPU restatement of StringSearch::StringIndex (nGramSearch.h:104)."""

    def __init__(self, words, row_size: int = 1, weights=None):
        L = lib()
        self._words = _words_array(words)  # keep alive during build
        w = None
        if weights is not None:
            w = (C.c_float * max(1, len(weights)))(*weights)
        self.h = L.ngo_build(self._words if words else None, len(words), row_size, w)
        self._keys: dict[int, bytes] = {}

    def close(self):
        if self.h:
            lib().ngo_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return lib().ngo_size(self.h)

    def lib_size(self) -> int:
        return lib().ngo_libsize(self.h)

    def n_keys(self) -> int:
        return lib().ngo_nkeys(self.h)

    def key(self, k: int) -> bytes:
        if k not in self._keys:
            n = C.c_uint32()
            p = lib().ngo_key(self.h, k, C.byref(n))
            self._keys[k] = C.string_at(p, n.value)
        return self._keys[k]

    def set_valid_char(self, chars) -> None:
        b = chars if isinstance(chars, bytes) else chars.encode("latin-1")
        lib().ngo_set_valid(self.h, b, len(b))

    def score_ids(self, query, threshold: float, limit: int):
        q = query if isinstance(query, bytes) else query.encode("latin-1")
        cap = max(1, min(limit if limit else 2**31 - 1, self.n_keys()))
        keys = (C.c_uint32 * cap)()
        scores = (C.c_float * cap)()
        n = lib().ngo_search(self.h, q, threshold, limit, keys, scores, cap)
        return list(keys[:n]), list(scores[:n])

    def score(self, query, threshold: float = 0.0, limit: int = 100):
        """Like dllmain.cpp:82 score(): list of (key bytes, fp32 score)."""
        ids, sc = self.score_ids(query, threshold, limit)
        return [(self.key(k), s) for k, s in zip(ids, sc)]

    def score_amb(self, query, threshold: float = 0.0, limit: int = 100):
        """score() plus whether the reference's answer depends on its unordered_map order beyond
        (score, length) ties (a promoted key with another pair above 100, ngs_oracle.c header)."""
        q = query if isinstance(query, bytes) else query.encode("latin-1")
        cap = max(1, min(limit if limit else 2**31 - 1, self.n_keys()))
        keys = (C.c_uint32 * cap)()
        scores = (C.c_float * cap)()
        amb = C.c_int(0)
        n = lib().ngo_search_amb(self.h, q, threshold, limit, keys, scores, cap, C.byref(amb))
        return [(self.key(k), s) for k, s in zip(keys[:n], scores[:n])], bool(amb.value)

    def score_batch(self, queries, threshold: float, limit: int, threads: int = 1):
        """Returns (counts[n], keys[n*cap], scores[n*cap], cap) as ctypes arrays."""
        n = len(queries)
        cap = max(1, min(limit if limit else 2**31 - 1, self.n_keys()))
        qs = (C.c_char_p * max(1, n))(*queries)
        counts = (C.c_uint32 * max(1, n))()
        keys = (C.c_uint32 * max(1, n * cap))()
        scores = (C.c_float * max(1, n * cap))()
        lib().ngo_search_batch(self.h, qs, n, threshold, limit, counts, keys, scores, cap, threads)
        return counts, keys, scores, cap


# ---- gram-size / UTF-32 restatement (libngs_oracle_g.so) -------------------------------
LIB_G_PATH = os.path.join(HERE, "libngs_oracle_g.so")
_lib_g = None
_U32P = C.POINTER(C.c_uint32)


def lib_g():
    global _lib_g
    if _lib_g is None:
        if not os.path.exists(LIB_G_PATH):
            build()
        L = C.CDLL(LIB_G_PATH)
        L.ngog_build.restype = C.c_void_p
        L.ngog_build.argtypes = [C.POINTER(_U32P), C.c_uint64, C.c_uint16, C.POINTER(C.c_float), C.c_uint32,
                                 C.c_int]
        L.ngog_free.argtypes = [C.c_void_p]
        L.ngog_size.restype = C.c_uint64
        L.ngog_size.argtypes = [C.c_void_p]
        L.ngog_libsize.restype = C.c_uint64
        L.ngog_libsize.argtypes = [C.c_void_p]
        L.ngog_nkeys.restype = C.c_uint32
        L.ngog_nkeys.argtypes = [C.c_void_p]
        L.ngog_key.restype = _U32P
        L.ngog_key.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.ngog_set_valid.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
        L.ngog_search.restype = C.c_uint32
        L.ngog_search.argtypes = [C.c_void_p, _U32P, C.c_float, C.c_uint32, C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_float), C.c_uint32]
        L.ngog_search_batch.argtypes = [C.c_void_p, C.POINTER(_U32P), C.c_uint32, C.c_float, C.c_uint32,
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_float),
                                        C.c_uint32, C.c_int]
        _lib_g = L
    return _lib_g


def _units(s):
    if isinstance(s, str):
        return [ord(c) for c in s]
    return [int(c) & 0xFFFFFFFF for c in s]  # bytes or a sequence of ints


def _u32(s):
    u = _units(s)
    return (C.c_uint32 * (len(u) + 1))(*u, 0)


class OracleIndexG:
    """Gram-size-g restatement. wide=False: byte strings (indexG semantics; g=3 is indexN);
    wide=True: UTF-32 strings (indexW semantics). Keys come back as str (wide) or bytes."""

    def __init__(self, words, row_size: int = 1, weights=None, g: int = 3, wide: bool = False):
        L = lib_g()
        self.wide = wide
        arrs = [None if w is None else _u32(w) for w in words]
        ptrs = (_U32P * max(1, len(words)))(*[None if a is None else C.cast(a, _U32P) for a in arrs])
        w = None
        if weights is not None:
            w = (C.c_float * max(1, len(weights)))(*weights)
        self.h = L.ngog_build(ptrs if words else None, len(words), row_size, w, g, int(wide))
        self._keys = {}

    def close(self):
        if self.h:
            lib_g().ngog_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return lib_g().ngog_size(self.h)

    def lib_size(self) -> int:
        return lib_g().ngog_libsize(self.h)

    def n_keys(self) -> int:
        return lib_g().ngog_nkeys(self.h)

    def key(self, k: int):
        if k not in self._keys:
            n = C.c_uint32()
            p = lib_g().ngog_key(self.h, k, C.byref(n))
            u = p[:n.value]
            self._keys[k] = "".join(map(chr, u)) if self.wide else bytes(u)
        return self._keys[k]

    def set_valid_char(self, chars) -> None:
        b = chars if isinstance(chars, bytes) else chars.encode("latin-1")
        lib_g().ngog_set_valid(self.h, b, len(b))

    def score(self, query, threshold: float = 0.0, limit: int = 100):
        cap = max(1, min(limit if limit else 2**31 - 1, self.n_keys()))
        keys = (C.c_uint32 * cap)()
        scores = (C.c_float * cap)()
        n = lib_g().ngog_search(self.h, C.cast(_u32(query), _U32P), threshold, limit, keys, scores, cap)
        return [(self.key(k), s) for k, s in zip(keys[:n], scores[:n])]

    def score_batch_raw(self, queries, threshold: float, limit: int, threads: int = 1):
        """Returns (counts[n], keys[n*cap], scores[n*cap], cap) as ctypes arrays."""
        n = len(queries)
        cap = max(1, min(limit if limit else 2**31 - 1, self.n_keys()))
        arrs = [_u32(q) for q in queries]
        qs = (_U32P * max(1, n))(*[C.cast(a, _U32P) for a in arrs])
        counts = (C.c_uint32 * max(1, n))()
        keys = (C.c_uint32 * max(1, n * cap))()
        scores = (C.c_float * max(1, n * cap))()
        lib_g().ngog_search_batch(self.h, qs, n, threshold, limit, counts, keys, scores, cap, threads)
        return counts, keys, scores, cap
