"""Diagnostic: index placement time with 1..R replicas (all on device 0 of a one-GPU box, the
replica threads contending for one GPU and one PCIe link as eight would for eight) at a BASELINE
config, for the C5 x 8 placement estimate in DESIGN.md §7. Prints per replica count the wall time
of indexN and the digest of every replica.
usage: python tools/placement_probe.py [rows=50000000] [max_replicas=3]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (imports torch first)
from stringsearchlib_amd import _native  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    t = time.time()
    corpus = bench.Corpus(rows)
    print(f"corpus {rows} rows generated in {time.time() - t:.1f} s", flush=True)
    L = _native.lib()
    for r in range(1, reps + 1):
        devs = (C.c_int * r)(*([0] * r))
        assert L.ngsSetDevices(devs, r) == 0
        t = time.time()
        h = L.indexN(corpus.words, corpus.n_words, corpus.row_size, corpus.weights)
        dt = time.time() - t
        assert h
        dig = []
        for i in range(r):
            d = (C.c_uint64 * 17)()
            assert L.ngsReplicaDigest(h, i, d, 17) == 17
            dig.append(tuple(d))
        same = all(x == dig[0] for x in dig)
        print(f"{r} replica(s): indexN {dt:.2f} s, replicas identical: {same}", flush=True)
        L.dispose(h)


if __name__ == "__main__":
    main()
