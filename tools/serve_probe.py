"""Diagnostic: score() latency with and without the server kernel (ngsServe) at a library size
(default the C3 10M rows): one query per call over the bench's query stream.
usage: python tools/serve_probe.py [rows=10000000] [calls=300]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (imports torch first)
from stringsearchlib_amd import _native  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    L = _native.lib()
    corpus = bench.Corpus(rows)
    h = bench.build_index(corpus, True, 0)
    raw, offs = corpus.queries(256)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(256)]
    res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()

    def timed():
        lat = []
        for i in range(n + 10):
            t = time.perf_counter()
            L.score(h, qs[i % 256], C.byref(res), C.byref(sc), 0.3, 100)
            lat.append(time.perf_counter() - t)
            L.release(h, res, sc)
        lat = sorted(lat[10:])
        return round(sum(lat) / len(lat) * 1e6, 1), round(lat[len(lat) // 2] * 1e6, 1)

    print(f"rows {rows}: score() mean/p50 us {timed()}", flush=True)
    assert L.ngsServe(h, 1) == 0
    print(f"rows {rows}: served score() mean/p50 us {timed()}", flush=True)
    L.ngsServe(h, 0)
    L.dispose(h)


if __name__ == "__main__":
    main()
