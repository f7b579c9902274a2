"""Run by test_gpu_arena.py in a process of its own with NGS_ECAP_INIT=256 (read once per process):
contexts start with 256 survivor slots per query, and 12-character queries over an 8-letter
library (cmin 3: the main tier-1a launch) have a few thousand survivors each, so every query goes
on in the batch's survivor arena. Call 1 of 1,024 queries runs the arena (1,024 blocks of 1,024)
out: those queries go to tier 1b and the arena grows; call 2 fits. Every answer must equal the
oracle's. Prints one JSON line."""
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
    rng = random.Random(60014)
    alphabet = b"ABCDEFGH"
    words = [bytes(rng.choice(alphabet) for _ in range(rng.randint(12, 30))) for _ in range(200000)]
    wts = [0.5 + rng.random() / 2 for _ in words]
    gi = ssl.StringIndex(words, 1, wts)
    gi.set_timing(True)
    oi = OracleIndex(words, 1, wts)
    qs = []
    for _ in range(1024):
        src = rng.choice(words)
        o = rng.randrange(len(src) - 11)
        q = bytearray(src[o:o + 12])
        q[rng.randrange(12)] = src[0]
        qs.append(bytes(q))
    sample = list(range(0, 1024, 16))
    refs = {i: oi.score(qs[i], 0.3, 100) for i in sample}
    fails, stats = [], []
    for call in range(3):
        got = gi.score_batch(qs, 0.3, 100)
        st = gi.last_stats()
        stats.append({k: st[k] for k in ("survivor_slots", "slot_full_queries", "handover_queries", "arena_blocks",
                                          "arena_used", "survivors", "fast_queries", "heavy_queries")})
        for i in sample:
            g, ref = got[i], refs[i]
            if len(g) != len(ref) or any(k1 != k2 or bits(s1) != bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)):
                fails.append(f"call {call} q#{i} {qs[i]!r}: {g[:3]} vs {ref[:3]}")
    # a smaller batch through the grown arena, every answer checked
    small = qs[:48]
    got = gi.score_batch(small, 0.3, 100)
    for i, (q, g) in enumerate(zip(small, got)):
        ref = oi.score(q, 0.3, 100)
        if len(g) != len(ref) or any(k1 != k2 or bits(s1) != bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)):
            fails.append(f"small q#{i} {q!r}: {g[:3]} vs {ref[:3]}")
    stats.append({k: gi.last_stats()[k] for k in ("arena_used", "slot_full_queries")})
    print(json.dumps({"fails": fails[:10], "stats": stats}))


if __name__ == "__main__":
    main()
