"""Run by test_gpu_slots.py in a process of its own with NGS_ECAP_INIT=256 (read once per process; the least it takes):
contexts start with 256 survivor slots per query, so a corpus with 259-712 survivors per
query fills them; the later calls must run with more slots, and every call's answer must equal
the oracle's. Prints one JSON line."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

import torch  # noqa: E402,F401  (one HIP runtime: torch first)

from oracle_py import OracleIndex  # noqa: E402
from tiecheck import bits  # noqa: E402

import stringsearchlib_amd as ssl  # noqa: E402


def main():
    rng = random.Random(60012)
    alphabet = b"ABCDEFGHIJKL"
    words = [bytes(rng.choice(alphabet) for _ in range(rng.randint(10, 30))) for _ in range(60000)]
    wts = [0.5 + rng.random() / 2 for _ in words]
    gi = ssl.StringIndex(words, 1, wts)
    gi.set_timing(True)
    oi = OracleIndex(words, 1, wts)
    qs = []
    for _ in range(48):  # 8 characters, 6 grams: thr 0.3 -> cmin 2, hundreds of survivors each
        src = rng.choice(words)
        o = rng.randrange(len(src) - 7)
        q = bytearray(src[o:o + 8])
        q[rng.randrange(8)] = src[0]
        qs.append(bytes(q))
    refs = [oi.score(q, 0.3, 100) for q in qs]
    fails, slots, full, handovers = [], [], [], []
    for call in range(6):
        got = gi.score_batch(qs, 0.3, 100)
        st = gi.last_stats()
        slots.append(st["survivor_slots"])
        full.append(st["slot_full_queries"])
        handovers.append(st["handover_queries"])
        for q, g, ref in zip(qs, got, refs):
            if len(g) != len(ref) or any(k1 != k2 or bits(s1) != bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)):
                fails.append(f"call {call} q={q!r}: {g[:3]} vs {ref[:3]}")
    # a context that ran a large batch, then small batches whose slots grow, must stay
    # within the 16 GiB slot budget (the rows are the batch's, not the large batch's); grown slots
    # go back after 16 calls in a row that fill none of them
    budget = 16 << 30
    light = [b"ZZZZZZZZ"] * 262144  # no gram of the library: no survivors, fast
    big = gi.score_batch(light, 0.3, 100)
    if any(big):
        fails.append("light batch returned results")
    bytes_seen = [gi.last_stats()["survivor_slot_bytes"]]
    for call in range(8):
        got = gi.score_batch(qs, 0.3, 100)
        st = gi.last_stats()
        slots.append(st["survivor_slots"])
        full.append(st["slot_full_queries"])
        bytes_seen.append(st["survivor_slot_bytes"])
        for q, g, ref in zip(qs, got, refs):
            if len(g) != len(ref) or any(k1 != k2 or bits(s1) != bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)):
                fails.append(f"regrow call {call} q={q!r}: {g[:3]} vs {ref[:3]}")
    calm_slots = []
    for call in range(40):
        gi.score_batch([b"ZZZZZZZZ"] * 48, 0.3, 100)
        calm_slots.append(gi.last_stats()["survivor_slots"])
    got = gi.score_batch(qs, 0.3, 100)  # still exact after the slots shrank
    for q, g, ref in zip(qs, got, refs):
        if len(g) != len(ref) or any(k1 != k2 or bits(s1) != bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)):
            fails.append(f"after shrink q={q!r}: {g[:3]} vs {ref[:3]}")
    if max(bytes_seen) > budget:
        fails.append(f"survivor slots past the budget: {bytes_seen}")
    print(json.dumps({"fails": fails[:10], "slots": slots, "slot_full": full, "handovers": handovers,
                      "bytes": bytes_seen, "calm_slots": calm_slots}))


if __name__ == "__main__":
    main()
