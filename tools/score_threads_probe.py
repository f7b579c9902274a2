"""Diagnostic: score() latency under concurrent callers at C1 (1k rows, threshold 0, limit 100),
with the server kernel (the default: score() starts it on a small library) and without it
(ngsServe(h, 0)). T threads each make N score() calls over the bench's query stream; prints the
per-call p50 / p90 latency and the calls per second of all threads together.
usage: python tools/score_threads_probe.py [calls per thread=300]"""
import ctypes as C
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (imports torch first)
from stringsearchlib_amd import _native  # noqa: E402


def run(L, h, qs, threads, calls):
    lat = [[] for _ in range(threads)]
    start = threading.Barrier(threads + 1)

    def worker(i):
        res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
        start.wait()
        for k in range(calls):
            q = qs[(i * calls + k) % len(qs)]
            t = time.perf_counter()
            L.score(h, q, C.byref(res), C.byref(sc), 0.0, 100)
            lat[i].append(time.perf_counter() - t)
            L.release(h, res, sc)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for th in ths:
        th.start()
    start.wait()
    t0 = time.perf_counter()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    all_l = sorted(x for l in lat for x in l)
    return statistics.median(all_l) * 1e6, all_l[int(0.9 * len(all_l))] * 1e6, threads * calls / el


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    corpus = bench.Corpus(1000)
    h = bench.build_index(corpus, False, 0)
    L = _native.lib()
    raw, offs = corpus.queries(4096)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(4096)]
    for mode in ("server", "no server"):
        if mode == "no server":
            L.ngsServe(h, 0)
        for threads in (1, 2, 4, 8):
            run(L, h, qs, threads, 20)  # warm
            p50, p90, rate = run(L, h, qs, threads, calls)
            print(f"{mode:9s} threads {threads}: p50 {p50:7.1f} us  p90 {p90:7.1f} us  {rate:9.0f} calls/s",
                  flush=True)
    L.dispose(h)


if __name__ == "__main__":
    main()
