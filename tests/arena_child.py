"""Run by test_gpu_arena.py in a process of its own with NGS_ECAP_INIT=256 and NGS_ARENA_INIT=256
(read once per process): contexts start with 256 survivor slots per query and an arena of 256 blocks
of 1,024. Random 30-character queries over a 1M-word, 15-letter library at threshold 0.1 (28 grams,
cmin 3: the main tier-1a launch) have ~1,900 survivors each, spread over ~300 parts (a few per part,
so the parts stay within the sketch's 64 candidates), so every query chains about two arena blocks.
Call 1 of 1,024 queries runs the arena out: the queries that find no block go to tier 1b and the
arena grows; call 2 fits. 64 of the queries are keys of the library (exact matches, promoted to 100
from the arena's survivors). With NGS_ARENA_INIT too large to allocate, every call runs without an
arena (its queries past their slots go to tier 1b). Every answer must equal the oracle's. Prints one
JSON line."""
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
    alphabet = b"ABCDEFGHIJKLMNO"
    words = [bytes(rng.choice(alphabet) for _ in range(rng.randint(18, 24))) for _ in range(1000000)]
    # 64 keys of 30 letters, queried exactly: ~1,900 survivors each (arena blocks) and an exact match,
    # promoted to 100 by k_emit's read-back of the arena (emit_query, the have_q path)
    exact = [bytes(rng.choice(alphabet) for _ in range(30)) for _ in range(64)]
    words += exact
    wts = [0.5 + rng.random() / 2 for _ in words]
    gi = ssl.StringIndex(words, 1, wts)
    gi.set_timing(True)
    oi = OracleIndex(words, 1, wts)
    qs = [bytes(rng.choice(alphabet) for _ in range(30)) for _ in range(1024 - len(exact))] + exact
    sample = list(range(0, 1024 - len(exact), 16)) + list(range(1024 - len(exact), 1024))
    refs = {i: oi.score(qs[i], 0.1, 100) for i in sample}
    fails, stats = [], []
    for call in range(3):
        got = gi.score_batch(qs, 0.1, 100)
        got_last = got
        st = gi.last_stats()
        stats.append({k: st[k] for k in ("survivor_slots", "slot_full_queries", "handover_queries", "arena_blocks",
                                          "arena_used", "survivors", "fast_queries", "heavy_queries")})
        for i in sample:
            g, ref = got[i], refs[i]
            if len(g) != len(ref) or any(k1 != k2 or bits(s1) != bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)):
                fails.append(f"call {call} q#{i} {qs[i]!r}: {g[:3]} vs {ref[:3]}")
    # a smaller batch through the grown arena, every answer checked
    small = qs[:48]
    got = gi.score_batch(small, 0.1, 100)
    for i, (q, g) in enumerate(zip(small, got)):
        ref = oi.score(q, 0.1, 100)
        if len(g) != len(ref) or any(k1 != k2 or bits(s1) != bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)):
            fails.append(f"small q#{i} {q!r}: {g[:3]} vs {ref[:3]}")
    stats.append({k: gi.last_stats()[k] for k in ("arena_used", "slot_full_queries")})
    promoted = sum(1 for i in range(1024 - len(exact), 1024) if got_last[i] and got_last[i][0][1] == 100.0)
    print(json.dumps({"fails": fails[:10], "stats": stats, "promoted": promoted, "exact": len(exact)}))


if __name__ == "__main__":
    main()
