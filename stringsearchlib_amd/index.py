"""Host-side mirror of the reference's interface (StringSearch::StringIndex + dllmain exports).

``StringIndex`` wraps one handle of libngram_search.so the way a host app drives the
reference DLL: ``indexN`` on construction (nGramSearch/dllmain.cpp:37), ``search`` /
``score`` (:61 / :82) returning master keys sorted by score, ``size`` / ``lib_size``
(:120 / :133), ``set_valid_char`` (:142) and ``dispose`` (:110). ``score_batch`` is the
batched extension that puts a whole query batch through one GPU pass.
"""
from __future__ import annotations

import ctypes as C

from . import _native

INT32_MAX = 2**31 - 1


def _b(s) -> bytes:
    return s if isinstance(s, bytes) else s.encode("latin-1")


class StringIndex:
    def __init__(self, words, row_size: int = 1, weights=None, device: int | None = None):
        L = _native.lib()
        if device is not None:
            rc = L.ngsSetDevice(device)
            if rc:
                raise RuntimeError(f"ngsSetDevice({device}) failed: {rc}")
        n = len(words)
        arr = (C.c_char_p * max(1, n))()
        for i, w in enumerate(words):
            arr[i] = None if w is None else _b(w)
        w = None
        if weights is not None:
            w = (C.c_float * max(1, len(weights)))(*weights)
        self.handle = L.indexN(arr if n else None, n, row_size, w)
        if not self.handle:
            raise RuntimeError("indexN failed (no usable GPU?) — see stderr")

    # -- reference exports -------------------------------------------------------------
    def size(self) -> int:
        return _native.lib().getSize(self.handle)

    def lib_size(self) -> int:
        return _native.lib().getLibSize(self.handle)

    def set_valid_char(self, chars) -> None:
        b = _b(chars)
        _native.lib().setValidChar(self.handle, b, len(b))

    def score(self, query, threshold: float = 0.0, limit: int = 100):
        """dllmain.cpp:82: list of (key bytes, fp32 score), best first."""
        L = _native.lib()
        res = C.POINTER(C.POINTER(C.c_char))()
        sc = C.POINTER(C.c_float)()
        n = L.score(self.handle, _b(query), C.byref(res), C.byref(sc), threshold, limit)
        if not n:
            if res:
                L.release(self.handle, res, sc)
            return []
        out = [(C.string_at(res[i]), sc[i]) for i in range(n)]
        L.release(self.handle, res, sc)
        return out

    def search(self, query, threshold: float = 0.0, limit: int = 100):
        """dllmain.cpp:61: list of key bytes, best first."""
        L = _native.lib()
        res = C.POINTER(C.POINTER(C.c_char))()
        n = L.search(self.handle, _b(query), C.byref(res), threshold, limit)
        out = [C.string_at(res[i]) for i in range(n)]
        if res:
            L.release(self.handle, res, None)
        return out

    def score_batch(self, queries, threshold: float = 0.0, limit: int = 100):
        """scoreBatch: one list of (key, score) per query."""
        L = _native.lib()
        nq = len(queries)
        qs = (C.c_char_p * max(1, nq))(*[_b(q) for q in queries])
        counts = (C.c_uint32 * max(1, nq))()
        res = C.POINTER(C.POINTER(C.c_char))()
        sc = C.POINTER(C.c_float)()
        total = L.scoreBatch(self.handle, qs, nq, threshold, limit, counts, C.byref(res), C.byref(sc))
        out, o = [], 0
        for i in range(nq):
            c = counts[i]
            out.append([(C.string_at(res[o + j]), sc[o + j]) for j in range(c)])
            o += c
        assert o == total
        if res:
            L.release(self.handle, res, sc)
        return out

    def dispose(self) -> None:
        if self.handle:
            _native.lib().dispose(self.handle)
            self.handle = 0

    def __del__(self):
        try:
            self.dispose()
        except Exception:
            pass

    # -- device-level extension ---------------------------------------------------------
    def num_keys(self) -> int:
        return _native.lib().ngsNumKeys(self.handle)

    def key(self, key_id: int) -> bytes:
        p = _native.lib().ngsKey(self.handle, key_id)
        if not p:
            raise IndexError(key_id)
        return C.string_at(p)

    def set_timing(self, enable: bool = True) -> None:
        _native.lib().ngsSetTiming(self.handle, int(enable))

    def last_stats(self) -> dict:
        st = _native.NgsStats()
        _native.lib().ngsLastStats(self.handle, C.byref(st))
        return {f: getattr(st, f) for f, _ in st._fields_}

    def search_device(self, d_bytes: int, d_offsets: int, n: int, threshold: float, limit: int, out_stride: int,
                      d_counts: int, d_keys: int, d_scores: int, stream: int = 0) -> None:
        """ngsSearchDevice on raw device pointers (e.g. torch tensors' data_ptr())."""
        rc = _native.lib().ngsSearchDevice(self.handle, d_bytes, d_offsets, n, threshold, limit, out_stride,
                                           d_counts, d_keys, d_scores, stream or None)
        if rc:
            raise RuntimeError(f"ngsSearchDevice failed: {rc}")
