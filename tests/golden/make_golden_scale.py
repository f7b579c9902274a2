"""Golden fixtures at the benchmark's own scale, from the REFERENCE implementation.

The small fixtures (make_golden.py) stop at 3,000 rows. These pin the path at BASELINE.json
configs[1] (C2: 1M rows, weight=NULL, threshold 0, limit 100) and configs[2] (C3: 10M rows,
per-row weights, threshold 0.3, limit 100): the reference DLL compiled from /root/reference
(oracle/Makefile) indexes the bench's own synthetic corpus (csrc/synth.c through
oracle/_ref/gen_golden's S record) and answers the first 256 queries of the bench's query
stream, plus, at C3, 16 rows' own keys (exact matches, promoted to 100).

A fixture stores the generator spec, not the corpus (the tests regenerate it with the same
generator), the queries, and per query the reference's count at the limit and its full
ranking (limit 0) cut after the (score, key length) class that holds the limit-th result:
enough for the tie-aware check (tests/tiecheck.py), whose boundary class is the only place
the reference's order is unspecified.

Measured in the build container (8 vCPU): C2 index 14 s, 2.4 GB RSS; C3 index ~180 s,
~18 GB RSS, 272 queries x 2 calls at ~0.14 s each.

    python tests/golden/make_golden_scale.py [c2] [c3]     # writes tests/golden/scale/*.json
"""
from __future__ import annotations

import json
import os
import resource
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from make_golden import GEN, REF_SO, fbits, hx  # noqa: E402

SYNTH = os.path.join(ROOT, "stringsearchlib_amd", "lib", "libngs_synth.so")
OUT = os.path.join(HERE, "scale")

SPECS = {
    "c2": dict(rows=1_000_000, seed=42, min_len=8, span=17, row_size=1, weights=False, thr=0.0, limit=100,
               n_queries=256, self_keys=0),
    "c3": dict(rows=10_000_000, seed=42, min_len=8, span=17, row_size=1, weights=True, thr=0.3, limit=100,
               n_queries=256, self_keys=16),
}


def queries(spec):
    """The bench's query stream (bench.Corpus over csrc/synth.c) and, optionally, rows' own keys."""
    import ctypes as C
    import bench
    corpus = bench.Corpus(spec["rows"], seed=spec["seed"], row_size=spec["row_size"])
    raw, offs = corpus.queries(spec["n_queries"])
    qs = [raw[offs[i]:offs[i + 1]] for i in range(spec["n_queries"])]
    step = max(1, spec["rows"] // max(1, spec["self_keys"]))
    for i in range(spec["self_keys"]):
        key = C.string_at(corpus.words[i * step * spec["row_size"]])
        qs.append(key if i % 2 == 0 else key.lower())  # lower case: same query after toUpper
    corpus.free()
    return qs


def cut_at_boundary(keys, scores, n):
    """The full ranking through the (score, key length) class of its n-th entry."""
    if n == 0 or n >= len(keys):
        return keys, scores
    last = (scores[n - 1], len(keys[n - 1]))
    end = n
    while end < len(keys) and (scores[end], len(keys[end])) == last:
        end += 1
    return keys[:end], scores[:end]


def build(name):
    spec = SPECS[name]
    qs = queries(spec)
    lines = [f"S {spec['rows']} {spec['seed']} {spec['min_len']} {spec['span']} {spec['row_size']} "
             f"{1 if spec['weights'] else 0} {SYNTH}"]
    for q in qs:
        lines.append(f"Q {hx(q) if q else '='} {fbits(spec['thr']):08x} {spec['limit']}")
        lines.append(f"Q {hx(q) if q else '='} {fbits(spec['thr']):08x} 0")
    lines.append("D")
    with tempfile.NamedTemporaryFile("w", suffix=".req", delete=False) as f:
        f.write("\n".join(lines) + "\n")
        req = f.name
    t0 = time.time()
    try:
        out = subprocess.run([GEN, REF_SO, req], check=True, capture_output=True, text=True)
    finally:
        os.unlink(req)
    rss = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss  # KiB, the largest child so far
    answers = [json.loads(l) for l in out.stdout.splitlines() if l.strip()]
    head, rest = answers[0], answers[1:]
    cases = []
    for i, q in enumerate(qs):
        a, full = rest[2 * i], rest[2 * i + 1]
        keys = [bytes.fromhex(k).decode("latin-1") for k in full["keys"]]
        fk, fs = cut_at_boundary(keys, full["scores"], a["n"])
        cases.append({"q": q.decode("latin-1"), "n": a["n"], "full_n": full["n"], "full_keys": fk, "full_scores": fs})
    fx = {"name": f"scale_{name}", "spec": spec, "size": head["size"], "libSize": head["libSize"],
          "reference_run": {"seconds": round(time.time() - t0, 1), "max_rss_kb": rss,
                            "driver": "oracle/_ref/gen_golden over oracle/_ref/libStringSearchLib.so"},
          "cases": cases}
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, f"{name}.json")
    with open(path, "w") as f:
        json.dump(fx, f, separators=(",", ":"))
    print(f"{path}: size={fx['size']} libSize={fx['libSize']} cases={len(cases)} "
          f"bytes={os.path.getsize(path)} ({fx['reference_run']})")


def main():
    if not (os.path.exists(REF_SO) and os.path.exists(GEN)):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    for name in sys.argv[1:] or ["c2", "c3"]:
        build(name)


if __name__ == "__main__":
    main()
