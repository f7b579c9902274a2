"""ctypes binding of libngram_search.so (include/ngram_search.h).

The library is built in-tree (``make -C stringsearchlib_amd/csrc``) and loaded from
``stringsearchlib_amd/lib``. There is no pure-Python or CPU fallback: if the library is
missing or no GPU is usable the calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import glob
import hashlib
import os
import re
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB_DIR = os.path.join(PKG, "lib")
# NGS_LIB=prof selects the phase-stamped diagnostic build (make -C csrc prof); NGS_LIB=<name>
# selects lib/libngram_search_<name>.so (experiment builds)
_variant = os.environ.get("NGS_LIB", "")
LIB_PATH = os.path.join(LIB_DIR, f"libngram_search_{_variant}.so" if _variant else "libngram_search.so")
SYNTH_PATH = os.path.join(LIB_DIR, "libngs_synth.so")
HEADER = os.path.join(ROOT, "include", "ngram_search.h")
CSRC = os.path.join(PKG, "csrc")


class NgsStats(C.Structure):
    _fields_ = [("queries", C.c_uint64), ("fast_queries", C.c_uint64), ("general_queries", C.c_uint64),
                ("postings", C.c_uint64), ("lists", C.c_uint64), ("results", C.c_uint64), ("survivors", C.c_uint64),
                ("fast_kernel_ms", C.c_double), ("prep_kernel_ms", C.c_double), ("general_ms", C.c_double),
                ("handover_queries", C.c_uint64), ("tier2_queries", C.c_uint64),
                ("heavy_queries", C.c_uint64), ("full_queries", C.c_uint64),
                ("slot_full_queries", C.c_uint64), ("survivor_slots", C.c_uint64),
                ("survivor_slot_bytes", C.c_uint64), ("main_postings", C.c_uint64), ("main_lists", C.c_uint64),
                ("arena_blocks", C.c_uint64), ("arena_used", C.c_uint64)]


def build(jobs: int = 4) -> None:
    """Compile the HIP library for gfx950 in-tree."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", CSRC], check=True)


_lib = None
_synth = None


def source_hash() -> str:
    """The stamp the Makefile bakes into ngsVersion(): SHA-256 (16 hex digits) of the library's
    sources (csrc/*.h, *.hip, *.cpp in byte order, then include/ngram_search.h)."""
    files = sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip")) +
                   glob.glob(os.path.join(CSRC, "*.cpp"))) + [HEADER]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` (HIP, gfx950)")
    L = C.CDLL(LIB_PATH)
    u32, u64, f32, cp = C.c_uint32, C.c_uint64, C.c_float, C.c_char_p
    PP = C.POINTER(C.POINTER(C.c_char))
    L.indexN.restype = u32
    L.indexN.argtypes = [C.POINTER(cp), u64, C.c_uint16, C.POINTER(f32)]
    L.search.restype = u32
    L.search.argtypes = [u32, cp, C.POINTER(PP), f32, u32]
    L.score.restype = u32
    L.score.argtypes = [u32, cp, C.POINTER(PP), C.POINTER(C.POINTER(f32)), f32, u32]
    L.release.restype = None
    L.release.argtypes = [u32, PP, C.POINTER(f32)]
    L.dispose.restype = None
    L.dispose.argtypes = [u32]
    L.getSize.restype = u64
    L.getSize.argtypes = [u32]
    L.getLibSize.restype = u64
    L.getLibSize.argtypes = [u32]
    L.setValidChar.restype = None
    L.setValidChar.argtypes = [u32, cp, C.c_int]
    L.scoreBatch.restype = u32
    L.scoreBatch.argtypes = [u32, C.POINTER(cp), u32, f32, u32, C.POINTER(u32), C.POINTER(PP),
                             C.POINTER(C.POINTER(f32))]
    L.searchBatch.restype = u32
    L.searchBatch.argtypes = [u32, C.POINTER(cp), u32, f32, u32, C.POINTER(u32), C.POINTER(PP)]
    # wide / gram-size extensions: wchar_t is 4 bytes on Linux, bound as uint32 units
    W = C.POINTER(C.c_uint32)
    PW = C.POINTER(W)
    L.indexG.restype = u32
    L.indexG.argtypes = [C.POINTER(cp), u64, C.c_uint16, C.POINTER(f32), C.c_uint16]
    L.indexW.restype = u32
    L.indexW.argtypes = [C.POINTER(W), u64, C.c_uint16, C.POINTER(f32), C.c_uint16]
    L.searchW.restype = u32
    L.searchW.argtypes = [u32, W, C.POINTER(PW), f32, u32]
    L.scoreW.restype = u32
    L.scoreW.argtypes = [u32, W, C.POINTER(PW), C.POINTER(C.POINTER(f32)), f32, u32]
    L.scoreBatchW.restype = u32
    L.scoreBatchW.argtypes = [u32, C.POINTER(W), u32, f32, u32, C.POINTER(u32), C.POINTER(PW),
                              C.POINTER(C.POINTER(f32))]
    L.searchBatchW.restype = u32
    L.searchBatchW.argtypes = [u32, C.POINTER(W), u32, f32, u32, C.POINTER(u32), C.POINTER(PW)]
    L.releaseW.restype = None
    L.releaseW.argtypes = [u32, PW, C.POINTER(f32)]
    L.disposeW.restype = None
    L.disposeW.argtypes = [u32]
    L.getSizeW.restype = u64
    L.getSizeW.argtypes = [u32]
    L.getLibSizeW.restype = u64
    L.getLibSizeW.argtypes = [u32]
    L.ngsKeyW.restype = C.c_void_p
    L.ngsKeyW.argtypes = [u32, u32]
    L.ngsCharSize.restype = u32
    L.ngsCharSize.argtypes = [u32]
    L.ngsGramSize.restype = u32
    L.ngsGramSize.argtypes = [u32]
    L.ngsSetDevice.restype = C.c_int
    L.ngsSetDevice.argtypes = [C.c_int]
    L.ngsSetDevices.restype = C.c_int
    L.ngsSetDevices.argtypes = [C.POINTER(C.c_int), C.c_int]
    L.ngsReplicaCount.restype = C.c_int
    L.ngsReplicaCount.argtypes = [u32]
    L.ngsDeviceCount.restype = C.c_int
    L.ngsDeviceCount.argtypes = []
    L.ngsNumKeys.restype = u32
    L.ngsNumKeys.argtypes = [u32]
    L.ngsKey.restype = C.c_void_p
    L.ngsKey.argtypes = [u32, u32]
    L.ngsSearchDevice.restype = C.c_int
    L.ngsSearchDevice.argtypes = [u32, C.c_void_p, C.c_void_p, u32, f32, u32, u32, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p]
    if hasattr(L, "ngsSearchDeviceAsync"):  # (experiment builds of older sources lack it)
        L.ngsSearchDeviceAsync.restype = C.c_int
        L.ngsSearchDeviceAsync.argtypes = [u32, C.c_void_p, C.c_void_p, u32, f32, u32, u32, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
        L.ngsSearchDeviceWait.restype = C.c_int
        L.ngsSearchDeviceWait.argtypes = [u32, C.c_uint64]
    if hasattr(L, "ngsServe"):
        L.ngsServe.restype = C.c_int
        L.ngsServe.argtypes = [u32, C.c_int]
    if hasattr(L, "ngsPackResults"):
        L.ngsPackResults.restype = C.c_int
        L.ngsPackResults.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, u32, u32, C.c_void_p, C.c_void_p, C.c_void_p]
    if hasattr(L, "ngsServeState"):
        L.ngsServeState.restype = C.c_int
        L.ngsServeState.argtypes = [u32]
    L.ngsSetTiming.restype = C.c_int
    L.ngsSetTiming.argtypes = [u32, C.c_int]
    if hasattr(L, "ngsLastError"):  # (experiment builds of older sources lack it)
        L.ngsLastError.restype = C.c_int
        L.ngsLastError.argtypes = [C.c_int]
    L.ngsLastStats.restype = C.c_int
    L.ngsLastStats.argtypes = [u32, C.POINTER(NgsStats)]
    L.ngsIndexDigest.restype = C.c_int
    L.ngsIndexDigest.argtypes = [u32, C.POINTER(u64), C.c_int]
    if hasattr(L, "ngsReplicaDigest"):
        L.ngsReplicaDigest.restype = C.c_int
        L.ngsReplicaDigest.argtypes = [u32, C.c_int, C.POINTER(u64), C.c_int]
    L.ngsVersion.restype = cp
    L.ngsVersion.argtypes = []
    L.ngsSaveIndex.restype = C.c_int
    L.ngsSaveIndex.argtypes = [u32, cp]
    L.ngsLoadIndex.restype = u32
    L.ngsLoadIndex.argtypes = [cp]
    L.ngsHostPhases.restype = C.c_int
    L.ngsHostPhases.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_int]
    L.ngsPhaseStats.restype = C.c_int
    L.ngsPhaseStats.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_int]
    version = L.ngsVersion().decode()
    want = source_hash()
    if not version.endswith(f"src={want}") and _variant:  # experiment builds (NGS_LIB) may predate the tree
        import sys
        print(f"[ngram_search] warning: {LIB_PATH} is {version!r}, the tree is src={want}", file=sys.stderr)
    elif not version.endswith(f"src={want}"):
        raise RuntimeError(f"{LIB_PATH} ({version!r}) was not built from this tree's sources (src={want}): "
                           f"rebuild it with `make -C {CSRC}`")
    _lib = L
    return L


def synth():
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise RuntimeError(f"{SYNTH_PATH} is missing: build it with `make -C {CSRC}`")
        S = C.CDLL(SYNTH_PATH)
        S.ngs_synth_corpus.restype = C.c_int
        S.ngs_synth_corpus.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                       C.POINTER(C.c_void_p), C.POINTER(C.POINTER(C.c_char_p)),
                                       C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_uint64)]
        S.ngs_synth_queries.restype = C.c_int
        S.ngs_synth_queries.argtypes = [C.POINTER(C.c_char_p), C.c_uint64, C.c_uint32, C.c_uint64,
                                        C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_void_p),
                                        C.POINTER(C.POINTER(C.c_uint64))]
        S.ngs_synth_free.restype = None
        S.ngs_synth_free.argtypes = [C.c_void_p]
        S.ngs_synth_widen.restype = C.c_int
        S.ngs_synth_widen.argtypes = [C.POINTER(C.c_char_p), C.c_uint64, C.POINTER(C.POINTER(C.c_uint32)),
                                      C.POINTER(C.POINTER(C.POINTER(C.c_uint32)))]
        _synth = S
    return _synth


def declared_symbols() -> list[str]:
    """Every function include/ngram_search.h declares with NGS_API."""
    text = open(HEADER).read()
    return re.findall(r"NGS_API\s+[\w\s\*]+?\b(\w+)\s*\(", text)
