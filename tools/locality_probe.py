"""Diagnostic: k_wave time on the C3 index when list reads hit cache vs when they do not.

Runs ngsSearchDevice on 65,536 queries in three orders:
  * "bench":  the benchmark stream (every query different, random lists);
  * "sorted": the same queries sorted by their normalised text (neighbours share grams);
  * "hot<k>": only k distinct queries, repeated (their lists stay in L2 / Infinity Cache).
The gap between "bench" and "hot" bounds what better list locality could buy.
usage: python tools/locality_probe.py [rows]
"""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402


def run(L, h, qs, thr=0.3, limit=100, reps=10):
    dev = torch.device("cuda", 0)
    raw = b"".join(qs)
    offs = [0]
    for q in qs:
        offs.append(offs[-1] + len(q))
    d_raw = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    B = len(qs)
    stride = limit
    d_cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    d_key = torch.zeros(B * stride, dtype=torch.int32, device=dev)
    d_sc = torch.zeros(B * stride, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    st = _native.NgsStats()
    L.ngsSetTiming(h, 1)
    ms = []
    for i in range(reps + 2):
        rc = L.ngsSearchDevice(h, d_raw.data_ptr(), d_off.data_ptr(), B, thr, limit, stride, d_cnt.data_ptr(),
                               d_key.data_ptr(), d_sc.data_ptr(), stream)
        assert rc == 0, rc
        L.ngsLastStats(h, C.byref(st))
        if i >= 2:
            ms.append(st.fast_kernel_ms)
    return sum(ms) / len(ms), st.postings / max(1, st.fast_queries)


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    torch.cuda.set_device(0)
    corpus = bench.Corpus(rows)
    h = bench.build_index(corpus, True, 0)
    L = _native.lib()
    B = 65536
    raw, offs = corpus.queries(B)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(B)]
    for name, batch in [("bench", qs), ("sorted", sorted(qs)), ("hot4096", [qs[i % 4096] for i in range(B)]),
                        ("hot256", [qs[i % 256] for i in range(B)]), ("hot32", [qs[i % 32] for i in range(B)]),
                        ("hot1", [qs[0]] * B)]:
        t = time.time()
        ms, ppq = run(L, h, batch)
        print(f"{name:8s} kernel {ms:7.3f} ms  {B / ms / 1e3:6.2f} Mq/s  postings/query {ppq:8.0f}  "
              f"({time.time() - t:.1f}s)", flush=True)
    L.dispose(h)


if __name__ == "__main__":
    main()
