"""Diagnostic: the cost of C3's heavy (cmin-2) queries on their own. Builds the C3 bench index and
times blocking ngsSearchDevice calls over (a) `n` of the bench's 12-character queries and (b) the
same queries cut to 8 characters (n = 6 grams, thr 0.3 -> cmin 2: every one on the heavy list).
Run it under rocprofv3 --kernel-trace to see the heavy chain's kernels alone.
usage: python tools/heavy_probe.py [n] [calls]"""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    corpus = bench.Corpus(10_000_000)
    h = bench.build_index(corpus, True, 0)
    L = _native.lib()
    L.ngsSetTiming(h, 1)
    raw, offs = corpus.queries(n)
    full = [raw[offs[i]:offs[i + 1]] for i in range(n)]
    dev = torch.device("cuda:0")
    for name, qs in (("qlen12", full), ("qlen8", [q[:8] for q in full])):
        blob = b"".join(qs)
        o = [0]
        for q in qs:
            o.append(o[-1] + len(q))
        d_raw = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        d_off = torch.tensor(o, dtype=torch.int64, device=dev)
        d_n = torch.zeros(n + 1, dtype=torch.int32, device=dev)
        d_k = torch.zeros(n * 100, dtype=torch.int32, device=dev)
        d_s = torch.zeros(n * 100, dtype=torch.float32, device=dev)
        ts = []
        for _ in range(calls):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rc = L.ngsSearchDevice(h, d_raw.data_ptr(), d_off.data_ptr(), n, C.c_float(0.3), 100, 100,
                                   d_n.data_ptr(), d_k.data_ptr(), d_s.data_ptr(), None)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
            if rc:
                raise RuntimeError(f"ngsSearchDevice -> {rc}")
        st = bench.last_stats(L, h) if hasattr(bench, "last_stats") else {}
        print(json.dumps({"set": name, "queries": n, "ms": [round(x, 3) for x in ts], "stats": st}), flush=True)


if __name__ == "__main__":
    main()
