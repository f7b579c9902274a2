"""Diagnostic: where a C2 step's host time goes (bench.py's pipelined loop, 3 batches in flight).

Times, per step, the host in ngsSearchDeviceAsync (queueing the call), in ngsSearchDeviceWait
(waiting for the oldest batch and finishing it) and in ngsLastStats, beside the step rate, with
depth 1, 2 and 3. usage: python tools/c2_host_probe.py [steps]
"""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    cfg = dict(bench.CONFIGS["c2"])
    dev = torch.device("cuda", 0)
    corpus = bench.Corpus(cfg["rows"])
    h = bench.build_index(corpus, cfg["weights"], 0, 3)
    L = _native.lib()
    B = cfg["batch"]
    raw, offs = corpus.queries(B)
    d_raw = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    stride = min(cfg["limit"], L.ngsNumKeys(h))
    L.ngsSetTiming(h, 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    bufs = [(torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B * stride, dtype=torch.int32, device=dev),
             torch.empty(B * stride, dtype=torch.float32, device=dev)) for _ in range(4)]
    st = _native.NgsStats()
    for depth in (1, 2, 3):
        inflight = []
        t_async = t_wait = t_stats = 0.0
        for k in range(steps + 20):
            if k == 20:
                torch.cuda.synchronize(dev)
                t_async = t_wait = t_stats = 0.0
                t0 = time.perf_counter()
            cnt, key, sc = bufs[k % 4]
            t = C.c_uint64()
            a = time.perf_counter()
            rc = L.ngsSearchDeviceAsync(h, d_raw.data_ptr(), d_off.data_ptr(), B, cfg["threshold"], cfg["limit"],
                                        stride, cnt.data_ptr(), key.data_ptr(), sc.data_ptr(), stream, C.byref(t))
            t_async += time.perf_counter() - a
            assert rc == 0, rc
            inflight.append(t.value)
            while len(inflight) >= depth:
                a = time.perf_counter()
                rc = L.ngsSearchDeviceWait(h, inflight.pop(0))
                b = time.perf_counter()
                L.ngsLastStats(h, C.byref(st))
                t_wait += b - a
                t_stats += time.perf_counter() - b
                assert rc == 0, rc
        while inflight:
            L.ngsSearchDeviceWait(h, inflight.pop(0))
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        us = 1e6 / steps
        print(f"depth {depth}: {el * us:7.1f} us/step ({B * steps / el / 1e6:5.2f} Mq/s); host per step: "
              f"async {t_async * us:6.1f} us, wait {t_wait * us:6.1f} us, stats {t_stats * us:5.1f} us, "
              f"rest {(el - t_async - t_wait - t_stats) * us:5.1f} us", flush=True)
    L.dispose(h)


if __name__ == "__main__":
    main()
