"""Diagnostic: average k_wave launch time (HIP events) on the C3 bench stream.
Used for ablations: NGS_DEBUG / NGS_LIB variants are read by the library at first use.
usage: python tools/kms.py [rows] [batch] [thr]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench  # noqa: E402
import locality_probe  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
    torch.cuda.set_device(0)
    corpus = bench.Corpus(rows)
    h = bench.build_index(corpus, True, 0)
    L = _native.lib()
    raw, offs = corpus.queries(B)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(B)]
    qlen = int(os.environ.get("KMS_QLEN", "0"))  # only queries of this length (heavy-query studies)
    if qlen:
        sel = [q for q in qs if len(q) == qlen]
        qs = [sel[i % len(sel)] for i in range(B)]
    ms, ppq = locality_probe.run(L, h, qs, thr=thr)
    st = _native.NgsStats()
    L.ngsLastStats(h, C.byref(st))
    print(f"NGS_DEBUG={os.environ.get('NGS_DEBUG', '0')} NGS_LIB={os.environ.get('NGS_LIB', '')} "
          f"rows={rows} B={B} thr={thr}: kernel {ms:.3f} ms, {B / ms / 1e3:.2f} Mq/s, postings/q {ppq:.0f}, "
          f"handover {st.handover_queries} tier2 {st.tier2_queries} general {st.general_queries}", flush=True)


if __name__ == "__main__":
    main()
