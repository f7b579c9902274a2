"""Throughput of the short-query paths (Levenshtein searchShort, nGramSearch.hpp:182-270) on a
library with many short terms: queries of 4-8 characters scan shortLib in tier 1b (one wave per
query), queries of <= 3 characters scan the whole library on the general path.
usage: [NGS_LIB=<variant>] python tools/short_bench.py [rows] [batch]"""
import ctypes as C
import os
import random
import sys
import time

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stringsearchlib_amd import _native  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    rng = random.Random(3)
    alpha = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"
    words = [bytes(rng.choice(alpha) for _ in range(rng.randint(3, 10))) for _ in range(rows)]
    L = _native.lib()
    arr = (C.c_char_p * rows)(*words)
    h = L.indexN(arr, rows, 1, None)
    short = [w for w in words if len(w) < 6]
    out = {"rows": rows, "short_terms": L.getSize(h) and len(set(short)), "version": L.ngsVersion().decode()}
    # m4-8: 4-8 characters (shortLib scan in tier 1b); mixed: the same draw before round 6, where a
    # 3-character source word gives a 3-character query (~1/8 of them) and so a whole-library scan
    cases = [("m4-8 (shortLib scan)", 4, 8, B, 4), ("m3-8 mixed (1/8 whole-library)", 4, 8, B, 0),
             ("m1-3 (whole-library scan)", 2, 3, 1024, 0)]
    for name, lo, hi, n, min_src in cases:
        pool = [w for w in words if len(w) >= min_src]
        qs = []
        for _ in range(n):
            src = rng.choice(pool)
            k = min(len(src), rng.randint(lo, hi))
            o = rng.randrange(len(src) - k + 1)
            qs.append(src[o:o + k])
        qa = (C.c_char_p * n)(*qs)
        counts = (C.c_uint32 * n)()
        res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
        L.scoreBatch(h, qa, n, 0.3, 100, counts, C.byref(res), C.byref(sc))
        L.release(h, res, sc)
        t = time.perf_counter()
        reps = 3
        for _ in range(reps):
            L.scoreBatch(h, qa, n, 0.3, 100, counts, C.byref(res), C.byref(sc))
            L.release(h, res, sc)
        dt = (time.perf_counter() - t) / reps
        out[name] = f"{n / dt:.0f} queries/s ({dt * 1e3:.1f} ms per {n})"
    print(out)
    L.dispose(h)


if __name__ == "__main__":
    main()
