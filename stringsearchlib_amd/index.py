"""Host-side mirror of the reference's interface (StringSearch::StringIndex + dllmain exports).

``StringIndex`` wraps one handle of libngram_search.so the way a host app drives the
reference DLL: ``indexN`` on construction (nGramSearch/dllmain.cpp:37), ``search`` /
``score`` (:61 / :82) returning master keys sorted by score, ``size`` / ``lib_size``
(:120 / :133), ``set_valid_char`` (:142) and ``dispose`` (:110). ``score_batch`` is the
batched extension that puts a whole query batch through one GPU pass.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _native

INT32_MAX = 2**31 - 1


def _b(s) -> bytes:
    return s if isinstance(s, bytes) else s.encode("latin-1")


# ngsLastError's codes that are not HIP errors (include/ngram_search.h)
NGS_ERR_INTERNAL = 0x10001
NGS_ERR_QUERY_BUFFER = 0x10002


def _check(what: str) -> None:
    """Raise if the last call on this thread failed (ngsLastError): the reference's entry points
    answer 0 on failure, which would otherwise read as "no results"."""
    e = _native.lib().ngsLastError(1)
    if e == NGS_ERR_INTERNAL:
        raise RuntimeError(f"{what} failed: a kernel reported an internal error (see stderr)")
    if e == NGS_ERR_QUERY_BUFFER:
        raise RuntimeError(f"{what} failed: the batch outgrew the normalised-query buffer")
    if e:
        raise RuntimeError(f"{what} failed: HIP error {e} (see stderr)")


class StringIndex:
    """One index of byte strings. gram_size 3 is the reference (indexN); 1 or 2 use the indexG
    extension (every reference threshold scaled by the gram size)."""

    def __init__(self, words, row_size: int = 1, weights=None, device: int | None = None, gram_size: int = 3,
                 devices=None):
        """devices: a list of HIP devices to place one replica of the index on each (ngsSetDevices;
        repeats allowed); batches are then split across the replicas."""
        L = _native.lib()
        if devices is not None:
            ds = (C.c_int * max(1, len(devices)))(*devices)
            rc = L.ngsSetDevices(ds, len(devices))
            if rc:
                raise RuntimeError(f"ngsSetDevices({list(devices)}) failed: {rc}")
        elif device is not None:
            rc = L.ngsSetDevice(device)
            if rc:
                raise RuntimeError(f"ngsSetDevice({device}) failed: {rc}")
        n = len(words)
        w = None
        if weights is not None:
            w = (C.c_float * max(1, len(weights)))(*weights)
        self.handle = 0
        try:
            self._keep = self._words(words)  # alive during the build only
            self.handle = self._index(L, self._keep if n else None, n, row_size, w, gram_size)
        finally:
            self._keep = None
            if devices is not None:  # the device list applies to this build only
                L.ngsSetDevices(None, 0)
        if not self.handle:
            raise RuntimeError(f"{self._INDEX} failed (no usable GPU, or gram_size not in 1..3?) — see stderr")

    def save(self, path) -> None:
        """Writes the index to `path` (ngsSaveIndex): the interned library; `load` rebuilds the
        rest on the GPU."""
        rc = _native.lib().ngsSaveIndex(self.handle, os.fsencode(path))
        if rc:
            raise OSError(f"ngsSaveIndex({path!r}) failed: {rc}")

    @classmethod
    def load(cls, path, devices=None):
        """An index from a file `save` wrote (ngsLoadIndex), of the same width as the saved one."""
        L = _native.lib()
        if devices is not None:
            ds = (C.c_int * max(1, len(devices)))(*devices)
            rc = L.ngsSetDevices(ds, len(devices))
            if rc:
                raise RuntimeError(f"ngsSetDevices({list(devices)}) failed: {rc}")
        try:
            handle = L.ngsLoadIndex(os.fsencode(path))
        finally:
            if devices is not None:
                L.ngsSetDevices(None, 0)
        if not handle:
            raise OSError(f"ngsLoadIndex({path!r}) failed: not an index file, or no usable GPU")
        cs = L.ngsCharSize(handle)
        if cs != cls._CS:
            L.dispose(handle)
            raise TypeError(f"{path!r} holds an index of {cs}-byte characters, not {cls.__name__}'s")
        self = cls.__new__(cls)
        self.handle = handle
        self._keep = None
        return self

    # -- per-width plumbing (overridden by WideStringIndex) ------------------------------
    _INDEX = "indexN"
    _CS = 1  # bytes per character

    @staticmethod
    def _words(words):
        arr = (C.c_char_p * max(1, len(words)))()
        for i, w in enumerate(words):
            arr[i] = None if w is None else _b(w)
        return arr

    @staticmethod
    def _index(L, arr, n, row_size, w, gram_size):
        if gram_size == 3:
            return L.indexN(arr, n, row_size, w)
        return L.indexG(arr, n, row_size, w, gram_size)

    _q = staticmethod(_b)
    _string = staticmethod(C.string_at)
    _RES = C.POINTER(C.POINTER(C.c_char))
    _fn = {"search": "search", "score": "score", "release": "release", "scoreBatch": "scoreBatch", "key": "ngsKey"}

    def _queries(self, queries):
        return (C.c_char_p * max(1, len(queries)))(*[_b(q) for q in queries])

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
        L, f = _native.lib(), self._fn
        res = self._RES()
        sc = C.POINTER(C.c_float)()
        L.ngsLastError(1)
        n = getattr(L, f["score"])(self.handle, self._q(query), C.byref(res), C.byref(sc), threshold, limit)
        if not n:
            _check(f["score"])
            if res:
                getattr(L, f["release"])(self.handle, res, sc)
            return []
        out = [(self._string(res[i]), sc[i]) for i in range(n)]
        getattr(L, f["release"])(self.handle, res, sc)
        return out

    def search(self, query, threshold: float = 0.0, limit: int = 100):
        """dllmain.cpp:61: list of key bytes, best first."""
        L, f = _native.lib(), self._fn
        res = self._RES()
        L.ngsLastError(1)
        n = getattr(L, f["search"])(self.handle, self._q(query), C.byref(res), threshold, limit)
        if not n:
            _check(f["search"])
        out = [self._string(res[i]) for i in range(n)]
        if res:
            getattr(L, f["release"])(self.handle, res, None)
        return out

    def score_batch(self, queries, threshold: float = 0.0, limit: int = 100):
        """scoreBatch: one list of (key, score) per query."""
        L, f = _native.lib(), self._fn
        nq = len(queries)
        qs = self._queries(queries)
        counts = (C.c_uint32 * max(1, nq))()
        res = self._RES()
        sc = C.POINTER(C.c_float)()
        L.ngsLastError(1)
        total = getattr(L, f["scoreBatch"])(self.handle, qs, nq, threshold, limit, counts, C.byref(res),
                                            C.byref(sc))
        if not total:
            _check(f["scoreBatch"])
        out, o = [], 0
        for i in range(nq):
            c = counts[i]
            out.append([(self._string(res[o + j]), sc[o + j]) for j in range(c)])
            o += c
        assert o == total
        if res:
            getattr(L, f["release"])(self.handle, res, sc)
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

    def key(self, key_id: int):
        p = getattr(_native.lib(), self._fn["key"])(self.handle, key_id)
        if not p:
            raise IndexError(key_id)
        return self._string(p)

    def replicas(self) -> int:
        """Devices the index was placed on (ngsReplicaCount)."""
        return _native.lib().ngsReplicaCount(self.handle)

    def gram_size(self) -> int:
        return _native.lib().ngsGramSize(self.handle)

    def serve(self, enable: bool = True) -> None:
        """ngsServe: single score()/search() calls through the persistent low-latency server (on a
        small library it also starts by itself after the 4th call; serve(False) turns that off)."""
        rc = _native.lib().ngsServe(self.handle, int(enable))
        if rc:
            raise RuntimeError(f"ngsServe failed: {rc}")

    def serve_state(self) -> int:
        """ngsServeState: 0 no server, 1 set up but its kernel stopped, 2 its kernel running."""
        return _native.lib().ngsServeState(self.handle)

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


    def search_device_async(self, d_bytes: int, d_offsets: int, n: int, threshold: float, limit: int,
                            out_stride: int, d_counts: int, d_keys: int, d_scores: int, stream: int = 0) -> int:
        """ngsSearchDeviceAsync: queues the search and returns its ticket (wait_device(ticket))."""
        t = C.c_uint64()
        rc = _native.lib().ngsSearchDeviceAsync(self.handle, d_bytes, d_offsets, n, threshold, limit, out_stride,
                                                d_counts, d_keys, d_scores, stream or None, C.byref(t))
        if rc:
            raise RuntimeError(f"ngsSearchDeviceAsync failed: {rc}")
        return t.value

    def wait_device(self, ticket: int) -> None:
        """ngsSearchDeviceWait: the results of that call are complete on return."""
        rc = _native.lib().ngsSearchDeviceWait(self.handle, ticket)
        if rc:
            raise RuntimeError(f"ngsSearchDeviceWait failed: {rc}")


# ---- wide strings (indexW extension) ---------------------------------------------------
_U32P = C.POINTER(C.c_uint32)


def _u32(s):
    """str (one unit per code point) or a sequence of ints -> NUL-terminated uint32 array."""
    units = [ord(c) for c in s] if isinstance(s, str) else [int(c) & 0xFFFFFFFF for c in s]
    return (C.c_uint32 * (len(units) + 1))(*units, 0)


def _wstring(p) -> str:
    """NUL-terminated UTF-32 string at p -> str (raises on units above 0x10FFFF)."""
    u = C.cast(p, _U32P)
    out = []
    i = 0
    while u[i]:
        out.append(chr(u[i]))
        i += 1
    return "".join(out)


class WideStringIndex(StringIndex):
    """indexW / searchW / scoreW (Readme.md:91,135): UTF-32 strings (Python str, or sequences
    of ints for raw code units such as values above 0x10FFFF), gram_size 1..3."""

    _INDEX = "indexW"
    _CS = 4
    _RES = C.POINTER(_U32P)
    _fn = {"search": "searchW", "score": "scoreW", "release": "releaseW", "scoreBatch": "scoreBatchW",
           "key": "ngsKeyW"}

    def __init__(self, words, row_size: int = 1, weights=None, device: int | None = None, gram_size: int = 2,
                 devices=None):
        super().__init__(words, row_size, weights, device, gram_size, devices)

    @staticmethod
    def _words(words):
        arrs = [None if w is None else _u32(w) for w in words]
        arr = (_U32P * max(1, len(words)))(*[None if a is None else C.cast(a, _U32P) for a in arrs])
        arr._arrs = arrs  # keep the strings alive with the pointer array
        return arr

    @staticmethod
    def _index(L, arr, n, row_size, w, gram_size):
        return L.indexW(arr, n, row_size, w, gram_size)

    @staticmethod
    def _q(query):
        return C.cast(_u32(query), _U32P)

    _string = staticmethod(_wstring)

    def _queries(self, queries):
        arrs = [_u32(q) for q in queries]
        arr = (_U32P * max(1, len(queries)))(*[C.cast(a, _U32P) for a in arrs])
        arr._arrs = arrs
        return arr

    def size(self) -> int:
        return _native.lib().getSizeW(self.handle)

    def lib_size(self) -> int:
        return _native.lib().getLibSizeW(self.handle)

    def dispose(self) -> None:
        if self.handle:
            _native.lib().disposeW(self.handle)
            self.handle = 0
