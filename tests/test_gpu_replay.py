"""Replayed one-stream calls (ngs_abi.cpp queue_search, Context::graphs): a batch whose queries are
all on the heavy list (threshold 0) and of at most kOneStreamBatch queries queues its kernels on one
stream; when a call repeats an earlier call's launch arguments, the sequence is built as a graph
(node by node, no stream capture) and replayed. The replay reads the query buffers as they are at
execution time, so different queries written into the same device buffers must give their own
answers, through the blocking ngsSearchDevice (on the caller's stream) and through the pipelined
ngsSearchDeviceAsync / ngsSearchDeviceWait (on a pooled context's stream), exact against the
oracle (nGramSearch.hpp:278-341, 397-401)."""
import ctypes as C
import random

import pytest

from oracle_py import OracleIndex
from test_gpu_parity import assert_exact

import stringsearchlib_amd as ssl
from stringsearchlib_amd import _native

pytestmark = pytest.mark.gpu


def _windows(rng, words, n, qlen=12):
    keys = [w for w in words if w and len(w) >= qlen]
    out = []
    for _ in range(n):
        src = rng.choice(keys)
        o = rng.randrange(len(src) - qlen + 1)
        q = bytearray(src[o:o + qlen])
        q[rng.randrange(qlen)] = ord(rng.choice("ABCDEFGHIJKLMNOPQRSTUVWXYZ"))
        out.append(bytes(q))
    return out


@pytest.mark.parametrize("weighted", [False, True])
def test_replayed_calls_read_their_own_queries(weighted):
    import torch
    words, wts, _ = ssl.synth.gen_corpus(20000, seed=31)
    wts = wts if weighted else None
    gi, oi = ssl.StringIndex(words, 1, wts), OracleIndex(words, 1, wts)
    rng = random.Random(5 + weighted)
    B, thr, limit = 200, 0.0, 50
    sets = [_windows(rng, words, B) for _ in range(3)]
    dev = torch.device("cuda", 0)
    d_raw = torch.empty(B * 12, dtype=torch.uint8, device=dev)
    d_off = torch.tensor([12 * i for i in range(B + 1)], dtype=torch.int64, device=dev)
    stride = limit
    d_cnt = torch.empty(B, dtype=torch.int32, device=dev)
    d_key = torch.empty(B * stride, dtype=torch.int32, device=dev)
    d_sc = torch.empty(B * stride, dtype=torch.float32, device=dev)
    L = _native.lib()
    side = torch.cuda.Stream(dev)  # (calls on the null stream are queued one by one, never replayed)
    stream = side.cuda_stream

    ph = (C.c_uint64 * 8)()
    L.ngsHostPhases(ph, 8, 1)

    def check(qs, where):
        cnt, key, sc = d_cnt.cpu().tolist(), d_key.cpu().tolist(), d_sc.cpu().tolist()
        for i, q in enumerate(qs):
            got = [(gi.key(key[i * stride + j]), sc[i * stride + j]) for j in range(cnt[i])]
            assert_exact(got, oi.score(q, thr, limit), f"{where} q={q!r}")

    # blocking calls: A B A B A C (the second A onward replays); the buffers are written on the
    # call's stream
    torch.cuda.synchronize(dev)
    for k, si in enumerate([0, 1, 0, 1, 0, 2]):
        with torch.cuda.stream(side):
            d_raw.copy_(torch.frombuffer(bytearray(b"".join(sets[si])), dtype=torch.uint8).to(dev))
            d_cnt.fill_(-1)
        gi.search_device(d_raw.data_ptr(), d_off.data_ptr(), B, thr, limit, stride, d_cnt.data_ptr(),
                         d_key.data_ptr(), d_sc.data_ptr(), stream)
        side.synchronize()
        check(sets[si], f"call {k} set {si}")
    L.ngsHostPhases(ph, 8, 1)
    assert ph[7] >= 3, list(ph)
    # pipelined, on a pooled context's stream: the second call builds the graph, the rest replay
    for k, si in enumerate([1, 2, 1, 2, 0, 1]):
        with torch.cuda.stream(side):
            d_raw.copy_(torch.frombuffer(bytearray(b"".join(sets[si])), dtype=torch.uint8).to(dev))
        t = C.c_uint64()
        assert L.ngsSearchDeviceAsync(gi.handle, d_raw.data_ptr(), d_off.data_ptr(), B, thr, limit, stride,
                                      d_cnt.data_ptr(), d_key.data_ptr(), d_sc.data_ptr(), stream, C.byref(t)) == 0
        assert L.ngsSearchDeviceWait(gi.handle, t.value) == 0
        side.synchronize()
        check(sets[si], f"async call {k} set {si}")
    L.ngsHostPhases(ph, 8, 1)
    assert ph[7] >= 3, list(ph)
    gi.dispose()
