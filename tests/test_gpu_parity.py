"""GPU path (libngram_search.so through its C ABI) against the reference and the oracle.

* every golden fixture: tie-aware against the REFERENCE's own answers, and exactly
  (keys, order, fp32 bits) against the CPU restatement, which uses the same tie refinement;
* seeded random corpora / queries covering every branch of the kernels (short Levenshtein
  scan, gram counting over several term-id parts, limits above the LDS top-k, general
  library-wide path, aliases, zero / negative weights, validChar changes): exact vs oracle;
* batch API == single-query API; device-pointer API == host API.
"""
import random
import zlib
import struct

import pytest

from conftest import fixture_weights, fixture_words, load_fixtures
from oracle_py import OracleIndex
from tiecheck import bits, check

import stringsearchlib_amd as ssl

pytestmark = pytest.mark.gpu
FIXTURES = load_fixtures()


def f32(b):
    return struct.unpack("<f", struct.pack("<I", b))[0]


def assert_exact(ours, ref, where):
    assert len(ours) == len(ref), f"{where}: {len(ours)} results vs oracle {len(ref)}\n{ours[:5]}\n{ref[:5]}"
    for i, ((k1, s1), (k2, s2)) in enumerate(zip(ours, ref)):
        assert k1 == k2 and bits(s1) == bits(s2), f"{where}: #{i} {k1!r}|{s1!r} vs oracle {k2!r}|{s2!r}"


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_fixture_parity(fx):
    words, weights = fixture_words(fx), fixture_weights(fx)
    gi = ssl.StringIndex(words, fx["rowSize"], weights)
    oi = OracleIndex(words, fx["rowSize"], weights)
    assert gi.size() == fx["size"]
    assert gi.lib_size() == fx["libSize"]
    for pi, ph in enumerate(fx["phases"]):
        if ph["validChar"] is not None:
            gi.set_valid_char(ph["validChar"].encode("latin-1"))
            oi.set_valid_char(ph["validChar"].encode("latin-1"))
        groups = {}
        for ci, c in enumerate(ph["cases"]):
            q, thr, limit = c["q"].encode("latin-1"), f32(c["thr"]), c["limit"]
            where = f"{fx['name']}[{pi}.{ci}] q={q!r} thr={thr} limit={limit}"
            ours = gi.score(q, thr, limit)
            check(ours, len(c["keys"]), c["full_keys"], c["full_scores"], where)
            assert_exact(ours, oi.score(q, thr, limit), where)
            assert gi.search(q, thr, limit) == [k for k, _ in ours]
            groups.setdefault((c["thr"], limit), []).append((q, ours))
        for (tb, limit), items in groups.items():
            batch = gi.score_batch([q for q, _ in items], f32(tb), limit)
            for (q, single), b in zip(items, batch):
                assert_exact(b, single, f"{fx['name']} batch q={q!r}")
    gi.dispose()


def _rand_queries(rng, words, n):
    alpha = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 abcxyz-#.%$@*\t"
    keys = [w for w in words if w]
    out = []
    for i in range(n):
        kind = i % 8
        src = rng.choice(keys)
        if kind == 0:      # bench-shaped: 12-byte window with one substitution
            l = min(12, len(src)); o = rng.randrange(len(src) - l + 1)
            q = bytearray(src[o:o + l]); q[rng.randrange(l)] = rng.choice(alpha[:26]); q = bytes(q)
        elif kind == 1:    # short substring (Levenshtein paths)
            l = rng.randint(1, min(8, len(src))); o = rng.randrange(len(src) - l + 1); q = src[o:o + l]
        elif kind == 2:    # exact key, maybe lower-cased (promotion)
            q = src if rng.random() < 0.5 else src.lower()
        elif kind == 3:    # random junk
            q = bytes(rng.choice(alpha) for _ in range(rng.randint(0, 20)))
        elif kind == 4:    # two keys glued (many grams, many candidates)
            q = src + b" " + rng.choice(keys)
        elif kind == 5:    # padded / escaped variants
            q = b"  " + src.replace(b" ", b"-") + b"!! "
        elif kind == 6:    # long query (> 257 bytes: general path)
            q = (src + b" ") * (300 // (len(src) + 1) + 1)
        else:              # window of 9..20 bytes
            l = min(len(src), rng.randint(9, 20)); o = rng.randrange(len(src) - l + 1); q = src[o:o + l]
        out.append(q)
    return out + [b"", b"*", b"   ", b"###"]


def _corpus(kind, rng):
    if kind == "bench":
        words, wts, _ = ssl.synth.gen_corpus(20000, seed=3)
        return words, 1, wts
    if kind == "short":
        words, _, _ = ssl.synth.gen_corpus(6000, seed=4, min_len=1, span=9)
        return words, 1, None
    if kind == "skewed":   # 4-letter alphabet: buckets above the part cap -> term-id sub-parts
        words = [bytes(rng.choice(b"ACGT") for _ in range(rng.randint(6, 30))) for _ in range(30000)]
        return words, 1, None
    if kind == "skew8":    # 8-letter alphabet: several bucket-range parts per query
        words = [bytes(rng.choice(b"ABCDEFGH") for _ in range(rng.randint(6, 30))) for _ in range(40000)]
        return words, 1, None
    if kind == "rows":     # aliases, NULL holes, zero / negative weights, duplicate keys
        words, wts, _ = ssl.synth.gen_corpus(3000, seed=9, min_len=3, span=12, row_size=3)
        words = list(words)
        for i in range(0, len(words), 29):
            words[i] = None
        for i in range(7, len(words), 31):
            words[i] = words[i - 6]
        for i in range(2, len(wts), 17):
            wts[i] = 0.0
        for i in range(4, len(wts), 19):
            wts[i] = -0.75
        return words, 3, wts
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["bench", "short", "skewed", "skew8", "rows"])
def test_random_parity_vs_oracle(kind):
    rng = random.Random(zlib.crc32(kind.encode()))
    words, rs, wts = _corpus(kind, rng)
    gi = ssl.StringIndex(words, rs, wts)
    oi = OracleIndex(words, rs, wts)
    assert gi.size() == oi.size() and gi.lib_size() == oi.lib_size()
    qs = _rand_queries(rng, [w for w in words if w], 48 if kind.startswith("skew") else 120)
    for thr, limit in [(0.0, 100), (0.3, 100), (0.5, 7), (0.0, 1), (0.25, 0), (1.0, 5), (0.0, 1500)]:
        got = gi.score_batch(qs, thr, limit)
        for q, g in zip(qs, got):
            assert_exact(g, oi.score(q, thr, limit), f"{kind} q={q!r} thr={thr} limit={limit}")
    gi.dispose()


def test_valid_char_changes_follow_oracle():
    words, wts, _ = ssl.synth.gen_corpus(2000, seed=12)
    gi, oi = ssl.StringIndex(words, 1, wts), OracleIndex(words, 1, wts)
    rng = random.Random(5)
    qs = _rand_queries(rng, words, 40)
    for valid in [b"ABCDEF ", b"0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ", bytes(range(1, 256))]:
        gi.set_valid_char(valid)
        oi.set_valid_char(valid)
        for q, g in zip(qs, gi.score_batch(qs, 0.2, 50)):
            assert_exact(g, oi.score(q, 0.2, 50), f"valid={valid[:8]!r} q={q!r}")


def test_device_api_matches_host_api():
    torch = pytest.importorskip("torch")
    words, wts, rng = ssl.synth.gen_corpus(5000, seed=21)
    qs = ssl.synth.gen_queries(words, 1, 300, rng) + [b"", b"*", b"AB"]
    gi = ssl.StringIndex(words, 1, wts)
    dev = torch.device("cuda:0")
    raw = torch.tensor(list(b"".join(qs)), dtype=torch.uint8, device=dev)
    offs = [0]
    for q in qs:
        offs.append(offs[-1] + len(q))
    off = torch.tensor(offs, dtype=torch.int64, device=dev)
    limit = 50
    counts = torch.zeros(len(qs), dtype=torch.int32, device=dev)
    keys = torch.zeros(len(qs) * limit, dtype=torch.int32, device=dev)
    scores = torch.zeros(len(qs) * limit, dtype=torch.float32, device=dev)
    gi.search_device(raw.data_ptr(), off.data_ptr(), len(qs), 0.3, limit, limit, counts.data_ptr(),
                     keys.data_ptr(), scores.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c, k, s = counts.cpu().tolist(), keys.cpu().tolist(), scores.cpu().tolist()
    host = gi.score_batch(qs, 0.3, limit)
    for i, h in enumerate(host):
        dv = [(gi.key(k[i * limit + j]), s[i * limit + j]) for j in range(c[i])]
        assert_exact(dv, h, f"device q={qs[i]!r}")


def test_device_async_api_matches_host_api():
    """ngsSearchDeviceAsync / ngsSearchDeviceWait: three batches in flight together (a limit-0
    one among them), each answered like the host API; unknown and reused tickets are refused."""
    torch = pytest.importorskip("torch")
    words, wts, rng = ssl.synth.gen_corpus(5000, seed=22)
    gi = ssl.StringIndex(words, 1, wts)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    batches = [ssl.synth.gen_queries(words, 1, n, rng) + [b"", b"*", b"AB"] for n in (300, 17, 120)]
    limit = 40
    calls = []
    for qs, lim in zip(batches, (limit, 0, limit)):
        raw = torch.tensor(list(b"".join(qs)), dtype=torch.uint8, device=dev)
        offs = [0]
        for q in qs:
            offs.append(offs[-1] + len(q))
        off = torch.tensor(offs, dtype=torch.int64, device=dev)
        stride = limit if lim else gi.num_keys()
        counts = torch.full((len(qs),), -1, dtype=torch.int32, device=dev)
        keys = torch.zeros(len(qs) * stride, dtype=torch.int32, device=dev)
        scores = torch.zeros(len(qs) * stride, dtype=torch.float32, device=dev)
        t = gi.search_device_async(raw.data_ptr(), off.data_ptr(), len(qs), 0.3, lim, stride, counts.data_ptr(),
                                   keys.data_ptr(), scores.data_ptr(), stream)
        calls.append((t, qs, lim, stride, counts, keys, scores, raw, off))
    for t, qs, lim, stride, counts, keys, scores, _, _ in reversed(calls):  # any order
        gi.wait_device(t)
        c, k, s = counts.cpu().tolist(), keys.cpu().tolist(), scores.cpu().tolist()
        host = gi.score_batch(qs, 0.3, lim)
        for i, h in enumerate(host):
            dv = [(gi.key(k[i * stride + j]), s[i * stride + j]) for j in range(c[i])]
            assert_exact(dv, h, f"async q={qs[i]!r} limit={lim}")
    with pytest.raises(RuntimeError):
        gi.wait_device(calls[0][0])  # already waited for
    with pytest.raises(RuntimeError):
        gi.wait_device(123456789)
    gi.dispose()


def test_device_api_query_buffer_grows():
    """ngsSearchDevice launches without reading the batch's byte count back once its context has a
    normalised-query buffer; a later, larger batch that does not fit is flagged by k_prep and the
    call reruns with a larger buffer (same answers as the host API)."""
    torch = pytest.importorskip("torch")
    words, wts, rng = ssl.synth.gen_corpus(5000, seed=23)
    gi = ssl.StringIndex(words, 1, wts)
    dev = torch.device("cuda:0")
    limit = 20

    def run(qs):
        raw = torch.tensor(list(b"".join(qs)), dtype=torch.uint8, device=dev)
        offs = [0]
        for q in qs:
            offs.append(offs[-1] + len(q))
        off = torch.tensor(offs, dtype=torch.int64, device=dev)
        counts = torch.zeros(len(qs), dtype=torch.int32, device=dev)
        keys = torch.zeros(len(qs) * limit, dtype=torch.int32, device=dev)
        scores = torch.zeros(len(qs) * limit, dtype=torch.float32, device=dev)
        gi.search_device(raw.data_ptr(), off.data_ptr(), len(qs), 0.3, limit, limit, counts.data_ptr(),
                         keys.data_ptr(), scores.data_ptr(), torch.cuda.current_stream().cuda_stream)
        c, k, s = counts.cpu().tolist(), keys.cpu().tolist(), scores.cpu().tolist()
        return [[(gi.key(k[i * limit + j]), s[i * limit + j]) for j in range(c[i])] for i in range(len(qs))]

    small = ssl.synth.gen_queries(words, 1, 50, rng)
    big = ssl.synth.gen_queries(words, 1, 200, rng) * 40 + [b"x" * 70000]  # > the first 64 KB buffer
    bigger = big + [b"y" * 400000]  # past the grown buffer too
    # (k_prep resets the statistics of a context whose last call left them clean, kPrepZero: a rerun
    # must leave them clean for the calls after it)
    for qs in (small, big, small, big, bigger, small):
        got = run(qs)
        host = gi.score_batch(qs, 0.3, limit)
        for i, h in enumerate(host):
            assert_exact(got[i], h, f"device q#{i} of {len(qs)}")
    gi.dispose()


def test_dispose_and_handle_reuse():
    words = [b"ALPHA BRAVO", b"CHARLIE DELTA", b"ECHO FOXTROT"]
    a = ssl.StringIndex(words)
    b = ssl.StringIndex(words)
    ha, hb = a.handle, b.handle
    a.dispose()
    c = ssl.StringIndex(words)
    assert c.handle == ha  # smallest free handle (dllmain.cpp:41-44)
    assert b.score(b"charlie delta", 0.3, 10)[0][0] == b"CHARLIE DELTA"
    b.dispose(); c.dispose()
    assert hb != ha
