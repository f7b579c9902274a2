"""Phase breakdown of the fused kernel (diagnostic build). Run with NGS_LIB=prof."""
import ctypes as C
import os
import sys
import time

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402

NAMES = ["init", "short", "grams", "btot", "plan", "skipld", "prefix", "insert", "extract", "loopend",
         "flush", "write"]


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
    corpus = bench.Corpus(rows)
    h = bench.build_index(corpus, True, 0)
    L = _native.lib()
    raw, offs = corpus.queries(B)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(B)]
    qlen = int(os.environ.get("KMS_QLEN", "0"))  # only queries of this length
    if qlen:
        sel = [q for q in qs if len(q) == qlen]
        qs = [sel[i % len(sel)] for i in range(B)]
    arr = (C.c_char_p * B)(*qs)
    counts = (C.c_uint32 * B)()
    for it in range(3):
        out = (C.c_uint64 * 32)()
        L.ngsPhaseStats(out, 32, 1)
        res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
        t = time.time()
        L.scoreBatch(h, arr, B, thr, 100, counts, C.byref(res), C.byref(sc))
        dt = time.time() - t
        L.release(h, res, sc)
        L.ngsPhaseStats(out, 32, 1)
    wn = ["setup+short", "grams", "dma-wait", "next_part", "issue", "sketch", "exact", "loop-exit", "emit",
          "flush", "write"]
    wt = sum(out[16 + i] for i in range(len(wn)))
    print(f"k_wave: per-query wave time {wt/B:.0f} cycles")
    for i, nm in enumerate(wn):
        print(f"  {nm:10s} {out[16+i]/B:9.0f} cyc/query  {100*out[16+i]/max(wt,1):5.1f} %")
    print(f"  parts/query {out[27]/B:.1f}  exact parts/query {out[28]/B:.2f}  sketch candidates/part "
          f"{out[29]/max(1, out[27]):.1f}  chunks/part {out[30]/max(1, out[27]):.1f}")
    tot = sum(out[i] for i in range(12))
    print(f"rows={rows} B={B} thr={thr} wall={dt*1e3:.1f} ms; per-query block time {tot/B/100:.2f} us")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:8s} {out[i]/B/100:9.2f} us/query  {100*out[i]/max(tot,1):5.1f} %")


if __name__ == "__main__":
    main()
