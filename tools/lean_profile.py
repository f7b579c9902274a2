"""Phase breakdown of the tier-1a lean kernel (diagnostic build: make -C stringsearchlib_amd/csrc prof,
then NGS_LIB=prof). Cycles (s_memtime) per query and phase, summed over the queries' waves, plus
part statistics. usage: NGS_LIB=prof python tools/lean_profile.py [rows] [batch] [thr] [qlen]"""
import ctypes as C
import os
import sys

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402

PHASES = ["setup+grams", "lane map", "plan (fast)", "plan (slow)", "stage", "sketch", "spill+exit"]


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
    qlen = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # > 0: queries cut to this many bytes (8: C3's heavy ones)
    corpus = bench.Corpus(rows)
    h = bench.build_index(corpus, True, 0)
    L = _native.lib()
    raw, offs = corpus.queries(B)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(B)]
    if qlen:
        qs = [q[:qlen] for q in qs]
    arr = (C.c_char_p * B)(*qs)
    counts = (C.c_uint32 * B)()
    out = (C.c_uint64 * 48)()
    for it in range(2):
        L.ngsPhaseStats(out, 48, 1)
        res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
        L.scoreBatch(h, arr, B, thr, 100, counts, C.byref(res), C.byref(sc))
        L.release(h, res, sc)
        L.ngsPhaseStats(out, 48, 1)
    st = _native.NgsStats()
    L.ngsLastStats(h, C.byref(st))
    # [32, 48): the main launch (lean_query_g, lane groups); [16, 32): the heavy list's (lean_query)
    for title, base, nq in (("main launch (lean_query_g)", 32, B - st.heavy_queries),
                            ("heavy list (lean_query)", 16, max(1, st.heavy_queries))):
        w = [out[base + i] for i in range(16)]
        tot = sum(w[:len(PHASES)])
        print(f"{title}: {nq} queries, {tot / nq:.0f} cycles per query (wave time)")
        for i, nm in enumerate(PHASES):
            print(f"  {nm:12s} {w[i] / nq:9.0f} cyc/query  {100 * w[i] / max(tot, 1):5.1f} %")
        parts = max(1, w[11])
        print(f"  parts/query {w[11] / nq:.1f}  slow-plan iterations/query {w[12] / nq:.2f}  rounds/part "
              f"{w[13] / parts:.2f}  candidates/part {w[14] / parts:.2f}  cold parts {100 * w[15] / parts:.0f} %")
        print(f"  per part: plan {(w[2] + w[3]) / parts:.0f}  stage {w[4] / parts:.0f}  sketch {w[5] / parts:.0f} cycles")


if __name__ == "__main__":
    main()
