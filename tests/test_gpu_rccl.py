"""The multi-GPU gather on the real collective library: bench.py's ranks hand their results to
rank 0 with one RCCL gather (`nccl` backend) of a fused device buffer (shard.GatherBuffer,
async, completed by PendingGather). The CPU tests cover the same code over gloo with two
ranks; the one-GPU box allows one RCCL rank, which still runs the nccl backend's gather, its
asynchronous work handle and the device-buffer decode end to end, on results the library wrote
into the buffer's views with ngsSearchDevice.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

import stringsearchlib_amd as ssl
from stringsearchlib_amd import shard

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_gather_of_device_results_one_rank():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        words, wts, rng = ssl.synth.gen_corpus(3000, seed=11)
        qs = ssl.synth.gen_queries(words, 1, 300, rng)
        gi = ssl.StringIndex(words, 1, wts)
        want = gi.score_batch(qs, 0.3, 16)
        flat = b"".join(qs)
        offs = [0]
        for q in qs:
            offs.append(offs[-1] + len(q))
        raw = torch.frombuffer(bytearray(flat), dtype=torch.uint8).to(dev)
        off = torch.tensor(offs, dtype=torch.int64, device=dev)
        stride = 16
        gb = shard.GatherBuffer(len(qs), stride, pad_b=len(qs) + 5, device=dev)
        stream = torch.cuda.current_stream().cuda_stream
        gi.search_device(raw.data_ptr(), off.data_ptr(), len(qs), 0.3, 16, stride, gb.counts.data_ptr(),
                         gb.keys.data_ptr(), gb.scores.data_ptr(), stream)
        pending = shard.gather_to_root(gb, async_op=True)
        pending.complete()  # the stream is ordered after the gather; the buffer may be rewritten
        (counts, keys, scores), = pending.wait()
        o = 0
        for i, w in enumerate(want):
            n = int(counts[i])
            got = [(gi.key(int(k)), float(s)) for k, s in zip(keys[o:o + n].tolist(), scores[o:o + n].tolist())]
            assert got == w, f"q#{i}"
            o += n
        assert o == keys.numel()
        # the packed form of bench.py's step loop: ngsPackResults on the device, then the gather of
        # the buffer's prefix up to a record capacity every rank holds (shard.GatherCap). Too small a
        # capacity first: the retired gather reads the all-reduced total (copied to pinned memory on a
        # side stream), gathers the buffer again whole and grows the capacity; then it fits
        pg = shard.PackedGather(len(qs), stride, pad_b=len(qs) + 5, device=dev)
        cap = shard.GatherCap(len(qs) + 5, stride, initial=8)
        for rnd in range(2):
            gi.search_device(raw.data_ptr(), off.data_ptr(), len(qs), 0.3, 16, stride, pg.counts.data_ptr(),
                             pg.keys.data_ptr(), pg.scores.data_ptr(), stream)
            pend = shard.gather_packed(pg.pack(ssl._native.lib().ngsPackResults, stream), async_op=True, cap=cap)
            sent = pend.words
            (pc, pk, ps), = pend.wait()
            assert torch.equal(pc, counts) and torch.equal(pk, keys) and torch.equal(ps.view(torch.int32),
                                                                                  scores.view(torch.int32))
            if rnd == 0:
                assert sent == 2 + len(qs) + 5 + 2 * 8 and pend.regathered and pend.words == 2 + len(qs) + 5 + 2 * o
                assert cap.regathers == 1 and cap.total >= o
            else:
                assert not pend.regathered and cap.regathers == 1 and sent == 2 + len(qs) + 5 + 2 * cap.total
        gi.dispose()
    finally:
        dist.destroy_process_group()
