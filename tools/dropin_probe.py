"""Diagnostic: scoreBatch (the drop-in batch path) on the C3 bench index, timed per call, for an
index with one replica and for one with R replicas on device 0 (ngsSetDevices: the batch is split
into R slices scored on the library's persistent replica workers, each in pointer mode, and joined
in the caller's arrays; replicas on one device split only with NGS_SPLIT_SAME_DEVICE=1, else the
first replica takes the batch). usage: [NGS_SPLIT_SAME_DEVICE=1] python tools/dropin_probe.py [calls] [replicas]"""
import ctypes as C
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (imports torch first)
from stringsearchlib_amd import _native  # noqa: E402


def build(corpus, replicas):
    L = _native.lib()
    ds = (C.c_int * replicas)(*([0] * replicas))
    if L.ngsSetDevices(ds, replicas):
        raise RuntimeError("ngsSetDevices failed")
    h = L.indexN(corpus.words, corpus.n_words, corpus.row_size, corpus.weights)
    L.ngsSetDevices(None, 0)
    assert h and L.ngsReplicaCount(h) == replicas
    return h


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    corpus = bench.Corpus(10_000_000)
    L = _native.lib()
    raw, offs = corpus.queries(65536)
    B = len(offs) - 1
    arr = (C.c_char_p * B)(*[raw[offs[i]:offs[i + 1]] for i in range(B)])
    counts = (C.c_uint32 * B)()
    res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
    out = {}
    for r in (1, reps):
        h = build(corpus, r)
        ms = []
        for i in range(calls + 2):
            t = time.perf_counter()
            n = L.scoreBatch(h, arr, B, 0.3, 100, counts, C.byref(res), C.byref(sc))
            t1 = time.perf_counter()
            L.release(h, res, sc)
            if i >= 2:
                ms.append((t1 - t) * 1e3)
        out[r] = (statistics.median(ms), min(ms), n)
        print(f"replicas={r}: scoreBatch of {B} queries p50 {out[r][0]:.2f} ms min {out[r][1]:.2f} ms "
              f"({n} results)", flush=True)
        L.dispose(h)
    print(f"{reps} replicas on one device against 1: {out[reps][0] / out[1][0]:.3f}x (p50)")


if __name__ == "__main__":
    main()
