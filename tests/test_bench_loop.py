"""bench.py's own multi-rank step loop (StepLoop) on CPU: world size 2 over gloo.

The library is replaced by a stand-in with the same entry points (ngsSearchDevice,
ngsSearchDeviceAsync / ngsSearchDeviceWait, ngsLastStats) that scores with the CPU oracle into the
buffers the loop hands it, so the loop itself runs as on the GPU box: gather buffers used in turn,
up to `depth` batches in flight, a batch's gather issued when it completes and ordered before its
buffer is rewritten (PendingGather.complete), the drain inside the timed region, the barriers and
the max-over-ranks elapsed time. Rank 0 decodes every gathered buffer of the timed steps and
checks each against the whole batch scored in one piece. The packed gathers start at a record
capacity below what the batches return (gather_cap), so the first ones overflow: they are
gathered again whole when retired and the capacity grows; the later ones fit.
"""
import ctypes as C
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle_py import OracleIndex
from stringsearchlib_amd import shard, synth

LIMIT = 16
THR = 0.25


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeLib:
    """The C ABI entry points StepLoop calls, over CPU tensors, answered by the oracle."""

    def __init__(self, oi, tensors, delay_s=0.0):
        self.oi, self.t = oi, {t.data_ptr(): t for t in tensors}
        self.jobs, self.next = {}, 1
        self.calls = {"sync": 0, "async": 0, "wait": 0}
        self.max_inflight = 0
        self.delay_s = delay_s

    def register(self, *ts):
        for t in ts:
            self.t[t.data_ptr()] = t

    def _run(self, raw, off, B, thr, limit, stride, cnt, keys, scores):
        data, offs = self.t[raw].numpy().tobytes(), self.t[off].tolist()
        c, k, s = self.t[cnt], self.t[keys], self.t[scores]
        for i in range(B):
            ids, sc = self.oi.score_ids(data[offs[i]:offs[i + 1]], thr, limit)
            c[i] = len(ids)
            k[i * stride:i * stride + len(ids)] = torch.tensor(ids, dtype=torch.int32)
            s[i * stride:i * stride + len(sc)] = torch.tensor(sc, dtype=torch.float32)

    def ngsSearchDevice(self, h, raw, off, B, thr, limit, stride, cnt, keys, scores, stream):
        self.calls["sync"] += 1
        self._run(raw, off, B, thr, limit, stride, cnt, keys, scores)
        return 0

    def ngsSearchDeviceAsync(self, h, raw, off, B, thr, limit, stride, cnt, keys, scores, stream, ticket):
        self.calls["async"] += 1
        t = self.next
        self.next += 1
        self.jobs[t] = (raw, off, B, thr, limit, stride, cnt, keys, scores)
        self.max_inflight = max(self.max_inflight, len(self.jobs))
        ticket._obj.value = t
        return 0

    def ngsSearchDeviceWait(self, h, t):
        self.calls["wait"] += 1
        if t not in self.jobs:
            return -3
        self._run(*self.jobs.pop(t))
        return 0

    def ngsLastStats(self, h, st):
        st._obj.fast_kernel_ms = 1.0
        return 0


def _worker(rank, world, port, depth, result_path, gather_cap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        words, wts, rng = synth.gen_corpus(2000, seed=3)
        queries = synth.gen_queries(words, 1, 40, rng)
        oi = OracleIndex(words, 1, wts)
        B = len(queries) // world  # each rank scores its own slice of the global stream
        mine = queries[rank * B:(rank + 1) * B]
        raw = torch.frombuffer(bytearray(b"".join(mine)), dtype=torch.uint8)
        offs = [0]
        for q in mine:
            offs.append(offs[-1] + len(q))
        off = torch.tensor(offs, dtype=torch.int64)
        fake = FakeLib(oi, [raw, off])
        loop = bench.StepLoop(fake, 1, raw, off, B, THR, LIMIT, LIMIT, depth, world, torch.device("cpu"), None,
                              gather_cap=gather_cap)
        for gb in loop.gbs:
            fake.register(gb.counts, gb.keys, gb.scores)
        loop.keep_gathers = True
        steps = 5
        elapsed, ktimes = loop.run(steps, warmup=2)
        assert len(ktimes) == steps and not fake.jobs and not loop.inflight and not loop.pending
        if depth > 1:
            assert fake.calls["async"] == steps + 2 and fake.calls["wait"] == steps + 2 and fake.calls["sync"] == 0
            assert fake.max_inflight == depth
        else:
            assert fake.calls["sync"] == steps + 2
        # the elapsed time is the max over ranks: every rank reports the same value
        e = torch.tensor([elapsed], dtype=torch.float64)
        mx = e.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        assert float(mx) == elapsed
        # the packed gather moves the records, not B x stride
        assert len(loop.gather_words) == steps
        assert all(w < 1 + B * (1 + 2 * LIMIT) for w in loop.gather_words), loop.gather_words
        if gather_cap is not None:  # the overflow path ran during the warm-up, then the capacity held
            assert loop.regathers_warmup >= 1 and loop.cap.total > gather_cap
            assert loop.cap.regathers == loop.regathers_warmup, (loop.cap.regathers, loop.regathers_warmup)
        if rank == 0:
            assert len(loop.gathered) == steps
            want = [tuple(map(list, oi.score_ids(q, THR, LIMIT))) for q in queries[:B * world]]
            ok = True
            for pg in loop.gathered:
                flat = []
                for counts, keys, scores in pg.wait():
                    o = 0
                    for n in counts.tolist():
                        flat.append((keys[o:o + n].tolist(), scores[o:o + n].tolist()))
                        o += n
                ok = ok and len(flat) == len(want) and all(
                    a == list(b[0]) and torch.equal(torch.tensor(sa, dtype=torch.float32),
                                                     torch.tensor(b[1], dtype=torch.float32))
                    for (a, sa), b in zip(flat, want))
            with open(result_path, "w") as f:
                f.write("ok" if ok else "mismatch")
        else:
            for pg in loop.gathered:
                assert pg.wait() is None
        oi.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("depth", [1, 2, 3])
@pytest.mark.parametrize("gather_cap", [None, 4])
def test_step_loop_two_ranks(tmp_path, depth, gather_cap):
    out = tmp_path / "result.txt"
    mp.spawn(_worker, args=(2, _free_port(), depth, str(out), gather_cap), nprocs=2, join=True)
    assert out.read_text() == "ok"
