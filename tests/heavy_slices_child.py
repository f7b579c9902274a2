"""Run by test_gpu_heavy_slices.py in a process of its own with NGS_HEAVY_SLICES set (read once per
process): the heavy list's launch splits every query into that many term-id slices, whatever the
lists' lengths, and the heavy-list parity cases of test_gpu_heavy.py and test_gpu_promotion.py must
still be exact against the oracle: slices sharing a query's survivor slots, the last one publishing
the count, hand-overs from any slice (one listing per query), rank-list queries, and a call with
more heavy items than its context's last one (the overflow launch). Prints "ok"."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

import torch  # noqa: E402,F401  (one HIP runtime: torch first)

import test_gpu_heavy as th  # noqa: E402
import test_gpu_promotion as tp  # noqa: E402


def hint_overflow():
    """A context's heavy launch takes as many workgroups as its last call had items; a call with
    more runs the rest in the overflow launch. 24 heavy queries, then 600, then 24 again on one
    index (one context), every answer exact."""
    import random
    from oracle_py import OracleIndex
    from tiecheck import bits
    import stringsearchlib_amd as ssl
    rng = random.Random(9090)
    words = th._words(rng, b"ABCDEFGHIJKL", 60000, 10, 30)
    wts = [0.5 + rng.random() / 2 for _ in words]
    gi = ssl.StringIndex(words, 1, wts)
    oi = OracleIndex(words, 1, wts)
    qs = th._queries(rng, words, 600)
    for batch in (qs[:24], qs, qs[100:124]):
        got = gi.score_batch(batch, 0.3, 100)
        for q, g in zip(batch, got):
            ref = oi.score(q, 0.3, 100)
            assert len(g) == len(ref) and all(k1 == k2 and bits(s1) == bits(s2) for (k1, s1), (k2, s2) in zip(g, ref)), \
                f"batch of {len(batch)} q={q!r}: {g[:3]} vs {ref[:3]}"
    gi.dispose()
    oi.close()


def main():
    hint_overflow()
    th.test_cmin2_spill_parity(b"ABCDEFGHIJKL", 60000, 10, 30, False)
    th.test_cmin2_spill_parity(b"ABCDEFGH", 40000, 6, 30, True)
    for weight in (None, 2.5):
        th.test_cmin1_rank_lists(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ", 60000, 8, 24, 12, weight)
    th.test_cmin1_rank_lists(b"ABC", 20000, 6, 20, 10, None)
    th.test_cmin1_ones_and_short_routing(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ", 60000, 8, 24, 12)
    for kind in ("pool_rows3", "uniform150"):
        tp.test_promotion_synthetic(kind)
    print("ok")


if __name__ == "__main__":
    main()
