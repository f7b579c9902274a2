"""Multi-device split behind the C ABI (ngsSetDevices, ngs_abi.cpp host_search).

An index built after ngsSetDevices holds one replica per listed device; scoreBatch/searchBatch cut
a batch of at least 4,096 queries per replica into contiguous slices, score them concurrently (one
host thread and stream per replica) and join them in query order. Queries are independent
(nGramSearch.hpp:372-470 scores each one on its own), so the joined answer must equal the one-device
answer exactly. A one-GPU box exercises the same code with several replicas on device 0.
"""
import ctypes as C

import pytest

from oracle_py import OracleIndex
from test_gpu_parity import assert_exact

import stringsearchlib_amd as ssl
from stringsearchlib_amd import _native

pytestmark = pytest.mark.gpu


def _digest(handle, replica):
    out = (C.c_uint64 * 17)()
    assert _native.lib().ngsReplicaDigest(handle, replica, out, 17) == 17
    return list(out)


def _corpus(n, seed):
    words, weights, rng = ssl.synth.gen_corpus(n, seed=seed)
    qs = ssl.synth.gen_queries(words, 1, 1024, rng)
    return words, weights, qs


@pytest.mark.parametrize("replicas", [2, 3])
def test_split_equals_single(replicas):
    words, weights, qs = _corpus(20000, 7 + replicas)
    batch = (qs * 13)[: 4096 * replicas + 517]  # every replica gets a slice; the last one is ragged
    one = ssl.StringIndex(words, 1, weights, device=0)
    multi = ssl.StringIndex(words, 1, weights, devices=[0] * replicas)
    assert one.replicas() == 1 and multi.replicas() == replicas
    assert multi.size() == one.size() and multi.lib_size() == one.lib_size()
    # the replicas after the first are placed concurrently (one host thread each): every one of
    # them holds exactly the arrays of the one-device index
    want = _digest(one.handle, 0)
    for r in range(replicas):
        assert _digest(multi.handle, r) == want, f"replica {r} differs"
    assert _native.lib().ngsReplicaDigest(multi.handle, replicas, (C.c_uint64 * 17)(), 17) == -1
    for thr, limit in [(0.3, 100), (0.0, 7), (0.5, 0)]:
        a = one.score_batch(batch, thr, limit)
        b = multi.score_batch(batch, thr, limit)
        assert len(a) == len(b) == len(batch)
        for i, (x, y) in enumerate(zip(a, b)):
            assert x == y, f"query #{i} {batch[i]!r} thr={thr} limit={limit}: split answer differs"
    # the split answer is also the reference answer (oracle sample across the slice borders)
    oi = OracleIndex(words, 1, weights)
    got = multi.score_batch(batch, 0.3, 100)
    for i in list(range(0, len(batch), 997)) + [4095, 4096, 4097, len(batch) - 1]:
        assert_exact(got[i], oi.score(batch[i], 0.3, 100), f"#{i} {batch[i]!r}")
    # a single query and a small batch stay on the first replica
    assert multi.score(batch[5], 0.3, 100) == one.score(batch[5], 0.3, 100)
    assert multi.score_batch(batch[:100], 0.3, 100) == one.score_batch(batch[:100], 0.3, 100)
    one.dispose()
    multi.dispose()


def test_device_list_applies_to_one_build():
    words, weights, _ = _corpus(3000, 11)
    multi = ssl.StringIndex(words, 1, weights, devices=[0, 0])
    after = ssl.StringIndex(words, 1, weights)
    assert multi.replicas() == 2 and after.replicas() == 1
    L = ssl._native.lib()
    import ctypes as C
    bad = (C.c_int * 1)(10_000)
    assert L.ngsSetDevices(bad, 1) < 0  # out-of-range device: refused, nothing changed
    assert ssl.StringIndex(words, 1, weights).replicas() == 1
    multi.dispose()
    after.dispose()
