"""Phase breakdown of the tier-1b full wave kernel (wave_query<1, false>) on a C2-shaped batch
(diagnostic build: make -C stringsearchlib_amd/csrc prof, then NGS_LIB=prof). s_memtime cycles per
query summed over its waves, by WSTAMP phase, plus parts and exact-pass counts.
usage: NGS_LIB=prof python tools/tier1b_profile.py [rows] [batch] [thr] [limit]"""
import ctypes as C
import os
import sys

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402

PHASES = ["short search", "grams", "take", "plan", "stage", "sketch/route", "exact count", "loop exit",
          "final emit", "final flush", "output"]


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    limit = int(sys.argv[4]) if len(sys.argv) > 4 else 100
    corpus = bench.Corpus(rows)
    h = bench.build_index(corpus, False, 0)
    L = _native.lib()
    raw, offs = corpus.queries(B)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(B)]
    arr = (C.c_char_p * B)(*qs)
    counts = (C.c_uint32 * B)()
    out = (C.c_uint64 * 32)()
    for _ in range(2):
        L.ngsPhaseStats(out, 32, 1)
        res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
        L.scoreBatch(h, arr, B, thr, limit, counts, C.byref(res), C.byref(sc))
        L.release(h, res, sc)
        L.ngsPhaseStats(out, 32, 1)
    w = [out[16 + i] for i in range(16)]
    tot = sum(w[:len(PHASES)])
    print(f"tier 1b: {tot / B:.0f} cycles per query (wave time)")
    for i, nm in enumerate(PHASES):
        print(f"  {nm:13s} {w[i] / B:9.0f} cyc/query  {100 * w[i] / max(tot, 1):5.1f} %")
    print(f"  parts/query {w[11] / B:.1f}  exact parts/query {w[12] / B:.1f}  entries/query {w[14] / B:.0f}")


if __name__ == "__main__":
    main()
