"""Diagnostic: scoreBatch (the drop-in batch path) on the C3 bench index, timed per call, with the
host batch pipelined in NGS_PIPE_CHUNKS chunks (read once per process; run one process per
setting). usage: NGS_PIPE_CHUNKS=4 python tools/dropin_probe.py [calls]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (imports torch first)
from stringsearchlib_amd import _native  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    corpus = bench.Corpus(10_000_000)
    h = bench.build_index(corpus, True, 0)
    L = _native.lib()
    raw, offs = corpus.queries(65536)
    B = len(offs) - 1
    arr = (C.c_char_p * B)(*[raw[offs[i]:offs[i + 1]] for i in range(B)])
    counts = (C.c_uint32 * B)()
    res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
    for i in range(calls):
        t = time.perf_counter()
        n = L.scoreBatch(h, arr, B, 0.3, 100, counts, C.byref(res), C.byref(sc))
        t1 = time.perf_counter()
        L.release(h, res, sc)
        print(f"chunks={os.environ.get('NGS_PIPE_CHUNKS', 'default')} call {i}: {(t1 - t) * 1e3:.2f} ms "
              f"({n} results)", flush=True)
    L.dispose(h)


if __name__ == "__main__":
    main()
