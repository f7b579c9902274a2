"""Run by test_gpu_term_order.py in a process of its own with NGS_TERM_ORDER=rank (the build
reads the variable once per process): term ids in key-rank order, so DevIndex.tk_monotone holds
and tier 1b raises its count threshold on score ties (raised_cmin in ngs_kernels.hip). Checks
the GPU build against the host build and every answer exactly against the oracle, whose term
ids stay in first-appearance order. Prints one JSON line."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

import ctypes as C  # noqa: E402

from oracle_py import OracleIndex  # noqa: E402
from tiecheck import bits  # noqa: E402

import stringsearchlib_amd as ssl  # noqa: E402
from stringsearchlib_amd import _native  # noqa: E402


def digest(idx):
    out = (C.c_uint64 * 17)()
    assert _native.lib().ngsIndexDigest(idx.handle, out, 17) == 17
    return list(out)


def main():
    fails, checked, flags = [], 0, []
    rng = random.Random(11)
    for name, rows, weighted, rs in [("unweighted", 20000, False, 1), ("weighted", 20000, True, 1),
                                     ("aliases", 6000, True, 3)]:
        words, wts, _ = ssl.synth.gen_corpus(rows, seed=rows + rs, row_size=rs)
        if not weighted:
            wts = None
        g = ssl.StringIndex(words, rs, wts)
        os.environ["NGS_HOST_INTERN"] = "1"
        h = ssl.StringIndex(words, rs, wts)
        del os.environ["NGS_HOST_INTERN"]
        dg, dh = digest(g), digest(h)
        flags.append(dg[16])
        if dg != dh:
            fails.append(f"{name}: device build {dg} vs host build {dh}")
        o = OracleIndex(words, rs, wts)
        keys = [w for w in words if w]
        qs = []
        for i in range(240):
            src = rng.choice(keys)
            l = min(rng.randint(4, 16), len(src))
            off = rng.randrange(len(src) - l + 1)
            qs.append(src[off:off + l] if i % 6 else src)
        for thr, limit in [(0.0, 100), (0.0, 10), (0.2, 50), (0.0, 1)]:
            got = g.score_batch(qs, thr, limit)
            for q, a in zip(qs, got):
                ref = o.score(q, thr, limit)
                checked += 1
                same = len(a) == len(ref) and all(k1 == k2 and bits(s1) == bits(s2)
                                                  for (k1, s1), (k2, s2) in zip(a, ref))
                if not same and len(fails) < 8:
                    fails.append(f"{name} q={q!r} thr={thr} limit={limit}: {a[:4]} vs {ref[:4]}")
        g.dispose()
        h.dispose()
    print(json.dumps({"fails": fails, "checked": checked, "flags": flags}))


if __name__ == "__main__":
    main()
