"""The reference's threading contract under concurrent callers (dllmain.cpp:22,39,63,84,100,112):
any number of threads may call search/score/release (shared lock) while indexN/dispose take the
lock exclusively; a dispose waits for the calls in flight on every handle.

Eight worker threads call score(), search() and scoreBatch() (batches of 1..300 queries, on both
sides of the 16-query latency-path cutoff) on two handles at once, every answer checked exactly
against the oracle; a ninth thread builds, queries and disposes indexes on further handles all the
while; a tenth turns the server kernel of handle A on and off (ngsServe) under the workers' score()
calls. Then handle B is disposed while the workers are still calling it: calls that finished
before the dispose started must be exact, later ones exact or empty, and nothing may crash. ctypes
releases the GIL for every foreign call, so the calls run concurrently in the library.
"""
import random
import threading
import time

import pytest

from oracle_py import OracleIndex
from tiecheck import bits

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu


def _same(got, ref):
    return len(got) == len(ref) and all(k1 == k2 and bits(s1) == bits(s2) for (k1, s1), (k2, s2) in zip(got, ref))


def _corpus(n, seed, weighted):
    words, weights, rng = ssl.synth.gen_corpus(n, seed=seed)
    qs = ssl.synth.gen_queries(words, 1, 400, rng)
    qs += [w for w in words[:8]] + [w.lower() for w in words[8:12]] + [w[:5] for w in words[12:16]]
    qs += [b"", b"*", b"AB", b"##"]
    return words, (weights if weighted else None), qs


def test_concurrent_calls_and_dispose():
    cases = [(0.3, 100), (0.0, 50), (0.5, 10)]
    sets = {}
    for name, (n, seed, weighted) in {"A": (1000, 11, False), "B": (20000, 12, True)}.items():
        words, weights, qs = _corpus(n, seed, weighted)
        oi = OracleIndex(words, 1, weights)
        ref = {(q, t, l): oi.score(q, t, l) for q in qs for t, l in cases}
        sets[name] = (words, weights, qs, ref)
    gA = ssl.StringIndex(sets["A"][0], 1, sets["A"][1])
    gB = ssl.StringIndex(sets["B"][0], 1, sets["B"][1])
    handles = {"A": gA, "B": gB}
    churn_words, _, churn_q = _corpus(3000, 13, False)
    churn_ref = OracleIndex(churn_words, 1, None).score(churn_q[0], 0.3, 100)

    fails, errors = [], []
    counts = {"calls": 0, "batch_queries": 0, "after_dispose_empty": 0}
    lock = threading.Lock()
    stop = threading.Event()       # the workers
    stop_side = threading.Event()  # the index churn and the ngsServe toggle
    dispose_started = [None]  # perf_counter when B's dispose began

    def record(msg):
        with lock:
            fails.append(msg)

    def worker(wid):
        rng = random.Random(1000 + wid)
        try:
            while not stop.is_set():
                name = rng.choice("AB")
                g = handles[name]
                words, weights, qs, ref = sets[name]
                t, l = rng.choice(cases)
                op = rng.random()
                if op < 0.4:
                    q = rng.choice(qs)
                    got = g.score(q, t, l)
                    want = [ref[(q, t, l)]]
                    res = [got]
                elif op < 0.6:
                    q = rng.choice(qs)
                    got = g.search(q, t, l)
                    want = [[k for k, _ in ref[(q, t, l)]]]
                    res = [[(k, 0.0) for k in got]]
                    want = [[(k, 0.0) for k in want[0]]]
                else:
                    nb = rng.choice([1, 5, 16, 17, 40, 300])
                    batch = [rng.choice(qs) for _ in range(nb)]
                    res = g.score_batch(batch, t, l)
                    want = [ref[(q, t, l)] for q in batch]
                t1 = time.perf_counter()
                ok = all(_same(r, w) for r, w in zip(res, want)) and len(res) == len(want)
                late = name == "B" and dispose_started[0] is not None and t1 >= dispose_started[0]
                if not ok:
                    if late and all(r == [] for r in res):
                        with lock:
                            counts["after_dispose_empty"] += 1
                    else:
                        bad = [i for i, (r, w) in enumerate(zip(res, want)) if not _same(r, w)]
                        i = bad[0] if bad else 0
                        qi = batch[i] if op >= 0.6 else q
                        record(f"worker {wid} {name} op {op:.2f} thr {t} limit {l} batch {len(res)} "
                               f"({len(bad)} wrong, first #{i} q={qi!r}): got {len(res[i])} {res[i][:4]} "
                               f"want {len(want[i])} {want[i][:4]}")
                with lock:
                    counts["calls"] += 1
                    if op >= 0.6:
                        counts["batch_queries"] += len(res)
        except Exception as e:  # noqa: BLE001
            errors.append(f"worker {wid}: {e!r}")

    def churn():
        try:
            while not stop_side.is_set():
                g = ssl.StringIndex(churn_words, 1, None)  # indexN takes the lock exclusively
                got = g.score(churn_q[0], 0.3, 100)
                if not _same(got, churn_ref):
                    record(f"churn index answer {got[:3]} vs {churn_ref[:3]}")
                g.dispose()
        except Exception as e:  # noqa: BLE001
            errors.append(f"churn: {e!r}")

    def toggle():
        try:
            on = True
            while not stop_side.is_set():
                gA.serve(on)
                on = not on
                time.sleep(0.01)
        except Exception as e:  # noqa: BLE001
            errors.append(f"toggle: {e!r}")

    workers = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    side = [threading.Thread(target=churn), threading.Thread(target=toggle)]
    for th in workers + side:
        th.start()
    time.sleep(6.0)
    # the side threads stop first (a freed handle number must not be reissued to the churn
    # thread while the workers still call B), then B is disposed under the workers' calls
    stop_side.set()
    for th in side:
        th.join(timeout=60)
    dispose_started[0] = time.perf_counter()
    hB = gB.handle
    gB.dispose()  # waits for B's calls in flight (exclusive lock)
    time.sleep(1.0)
    stop.set()
    for th in workers:
        th.join(timeout=60)
    assert not any(th.is_alive() for th in workers + side), "a thread did not finish"
    assert not errors, "\n".join(errors[:10])
    assert not fails, f"{len(fails)} wrong answers:\n" + "\n".join(fails[:10])
    assert counts["calls"] > 200 and counts["batch_queries"] > 1000, counts
    assert ssl._native.lib().getSize(hB) == 0  # B is gone
    # A still answers exactly after all of it
    words, weights, qs, ref = sets["A"]
    for q in qs[:50]:
        assert _same(gA.score(q, 0.3, 100), ref[(q, 0.3, 100)]), q
    gA.dispose()

