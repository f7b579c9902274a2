"""C4's survivor memory per call (diagnostic): the full C4 batch (bench.py's corpus) through
scoreBatchW several times, printing the tier-1a survivor totals, the arena's blocks and use, the
queries handed over for their slots and the context's survivor bytes. Slots per query from
NGS_ECAP_INIT (else the library's default). usage: python tools/c4_arena_probe.py [calls]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import torch  # noqa: F401,E402  (one HIP runtime: torch first)

import bench  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402
from test_gpu_c4c5 import gpu_batch_w  # noqa: E402


def main(calls):
    cfg = bench.CONFIGS["c4"]
    corpus4 = bench.Corpus(cfg["rows"], row_size=cfg["row_size"], wide=True)
    h = bench.build_index(corpus4, False, 0, gram=cfg["gram"])
    L = _native.lib()
    raw, offs = corpus4.queries(cfg["batch"])
    qs = [tuple(raw[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
    L.ngsSetTiming(h, 1)
    st = _native.NgsStats()
    for call in range(calls):
        t = time.perf_counter()
        gpu_batch_w(h, qs, cfg["threshold"], cfg["limit"], decode=[])
        dt = time.perf_counter() - t
        L.ngsLastStats(h, C.byref(st))
        print(f"ecap_init={os.environ.get('NGS_ECAP_INIT', '-')} call {call}: {dt * 1e3:8.1f} ms  "
              f"fast {st.fast_queries} heavy {st.heavy_queries} handover {st.handover_queries} "
              f"slot_full {st.slot_full_queries}  survivors {st.survivors}  slots {st.survivor_slots}  "
              f"arena {st.arena_used}/{st.arena_blocks}  bytes {st.survivor_slot_bytes / 2**20:.0f} MiB", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
