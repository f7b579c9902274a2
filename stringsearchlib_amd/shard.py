"""Query-batch sharding across GPUs.

Each rank (one process per GPU) holds a replica of the index and scores a contiguous slice
of the batch; the only collective is the gather of the top-k records to rank 0 (RCCL over
xGMI with the ``nccl`` backend; ``gloo`` in the CPU tests). Queries share no state, so
nothing else crosses ranks.

bench.py's step loop gathers packed records (PackedGather): a finished batch's results are
packed on the device (ngsPackResults: a prefix sum of the counts and one {key, score} pair per
record) and the gather moves [batch, total, counts, records] up to a record capacity every rank
already holds (GatherCap), so the bytes on xGMI follow the results (about 20 per query at C3)
instead of the output stride (100), with no host read in the step. An 8-byte all-reduce of the
batch's largest total travels beside the gather; when the gather is retired (its buffer is about
to be rewritten, a step or more later) every rank reads that total, and if it exceeded the
capacity the buffers are gathered again whole and the capacity grows. The gathers run on RCCL's
stream beside the next batch's kernels. GatherBuffer / gather_to_root are the fixed-size
form (no size agreement: batch x stride records per rank), kept for callers that hold tensors.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(rank: int, world: int, n: int) -> tuple[int, int]:
    """Contiguous slice [lo, hi) of n queries for `rank`."""
    return n * rank // world, n * (rank + 1) // world


def max_shard(world: int, n: int) -> int:
    """The largest slice shard_bounds gives any rank (the gather's padded batch)."""
    return max(hi - lo for lo, hi in (shard_bounds(r, world, n) for r in range(world)))


def compact(counts: torch.Tensor, keys: torch.Tensor, scores: torch.Tensor, stride: int):
    """(counts[B], keys[B*stride], scores[B*stride]) -> counts, packed keys, packed scores.
    Boolean-mask indexing reads the packed size back to the host: rank 0 uses it after the gather."""
    B = counts.numel()
    mask = torch.arange(stride, device=counts.device).unsqueeze(0) < counts.view(B, 1).to(torch.int64)
    return counts, keys.view(B, stride)[mask], scores.view(B, stride)[mask]


class GatherBuffer:
    """One rank's fused int32 gather buffer: [batch, counts[pad_b], keys[pad_b*stride],
    score bits[pad_b*stride]]. ``counts``, ``keys`` and ``scores`` (float32) are views of it in
    ngsSearchDevice's output layout (query i's records at i*stride)."""

    def __init__(self, batch: int, stride: int, pad_b: int | None = None, device=None):
        pad_b = batch if pad_b is None else pad_b
        if batch > pad_b:
            raise ValueError(f"batch {batch} > padded batch {pad_b}")
        self.batch, self.stride, self.pad_b = batch, stride, pad_b
        self.buf = torch.zeros(1 + pad_b * (1 + 2 * stride), dtype=torch.int32, device=device)
        self.buf[0] = batch
        ko = 1 + pad_b
        so = ko + pad_b * stride
        self.counts = self.buf[1:1 + batch]
        self.keys = self.buf[ko:ko + batch * stride]
        self.scores = self.buf[so:so + batch * stride].view(torch.float32)

    def fill(self, counts: torch.Tensor, keys: torch.Tensor, scores: torch.Tensor):
        """Copies results written elsewhere into the views (device copies, no host sync)."""
        self.counts.copy_(counts.to(torch.int32))
        self.keys.copy_(keys.to(torch.int32))
        self.scores.copy_(scores.to(torch.float32))
        return self

    @staticmethod
    def decode(buf: torch.Tensor, stride: int, pad_b: int):
        """(counts, packed keys, packed scores) of a gathered buffer."""
        b = int(buf[0])
        if not 0 <= b <= pad_b or buf.numel() != 1 + pad_b * (1 + 2 * stride):
            raise ValueError(f"gathered buffer of batch {b} / {buf.numel()} words does not match pad_b {pad_b}, "
                             f"stride {stride}")
        ko = 1 + pad_b
        so = ko + pad_b * stride
        return compact(buf[1:1 + b], buf[ko:ko + b * stride], buf[so:so + b * stride].view(torch.float32), stride)


class PendingGather:
    """An in-flight gather (``gather_to_root(..., async_op=True)``): ``wait()`` returns what the
    blocking call returns (the per-rank lists on rank 0, None elsewhere)."""

    def __init__(self, work, gb: GatherBuffer, bufs, rank):
        self.work, self.gb, self.bufs, self.rank = work, gb, bufs, rank

    def complete(self):
        """Orders the current stream after the gather (no host synchronisation, no decode): the
        buffer may be written again afterwards."""
        self.work.wait()

    def wait(self):
        self.work.wait()
        if self.rank != 0:
            return None
        return [GatherBuffer.decode(b, self.gb.stride, self.gb.pad_b) for b in self.bufs]


def gather_to_root(counts, keys=None, scores=None, stride: int | None = None, group=None, async_op: bool = False,
                   pad_b: int | None = None):
    """Gathers every rank's top-k records on rank 0 with one collective.

    ``counts`` is a GatherBuffer that ngsSearchDevice wrote into, or the (counts, keys, scores)
    tensors of its output layout with their ``stride`` (they are copied into a new buffer).
    Every rank must use the same ``pad_b`` and stride. Returns the per-rank (counts, packed keys,
    packed scores) on rank 0 and None elsewhere; with ``async_op`` the gather stays in flight
    (RCCL runs it on its own stream, beside the next batch's kernels) and a PendingGather is
    returned."""
    if isinstance(counts, GatherBuffer):
        gb = counts
    else:
        if stride is None:
            raise ValueError("stride is required with tensor arguments")
        if pad_b is None:
            # uneven slices (n % world != 0) give ranks different batch sizes, and dist.gather of
            # buffers of different lengths hangs or corrupts: agree on the largest one (one small
            # all-reduce; callers that know it pass pad_b, e.g. shard.max_shard)
            m = torch.tensor([counts.numel()], dtype=torch.int64, device=counts.device)
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
            pad_b = int(m.item())
        gb = GatherBuffer(counts.numel(), stride, pad_b, counts.device).fill(counts, keys, scores)
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    bufs = [torch.empty_like(gb.buf) for _ in range(world)] if rank == 0 else None
    work = dist.gather(gb.buf, bufs, dst=0, group=group, async_op=True)
    pending = PendingGather(work, gb, bufs, rank)
    return pending if async_op else pending.wait()


def pack_torch(counts, keys, scores, n, stride, offsets, records):
    """ngsPackResults over torch tensors (CPU tests; the GPU path calls the library): offsets[n + 1]
    = exclusive prefix sum of counts, records[2 * total] = {key, score bits} in query order."""
    c = counts[:n].to(torch.int64)
    offsets[0] = 0
    offsets[1:n + 1] = torch.cumsum(c, 0).to(offsets.dtype)
    mask = torch.arange(stride, device=counts.device).unsqueeze(0) < c.view(n, 1)
    k = keys[:n * stride].view(n, stride)[mask]
    sb = scores[:n * stride].view(n, stride)[mask].view(torch.int32)
    t = k.numel()
    rec = records[:2 * t].view(t, 2)
    rec[:, 0] = k
    rec[:, 1] = sb


class PackedGather:
    """One batch's results and its packed gather buffer. ngsSearchDevice writes ``counts`` (a view
    of the buffer), ``keys`` and ``scores`` (query i's records at i * stride); ``pack`` then fills the
    buffer's [batch, total, counts[pad_b], records[2 * total]] on the device; ``gather_packed`` sends
    its prefix up to the largest total over the ranks."""

    def __init__(self, batch: int, stride: int, pad_b: int | None = None, device=None):
        pad_b = batch if pad_b is None else pad_b
        if batch > pad_b:
            raise ValueError(f"batch {batch} > padded batch {pad_b}")
        self.batch, self.stride, self.pad_b = batch, stride, pad_b
        self.buf = torch.zeros(2 + pad_b + 2 * pad_b * stride, dtype=torch.int32, device=device)
        self.buf[0] = batch
        self.counts = self.buf[2:2 + batch]
        self.records = self.buf[2 + pad_b:]
        self.keys = torch.zeros(max(1, batch * stride), dtype=torch.int32, device=device)
        self.scores = torch.zeros(max(1, batch * stride), dtype=torch.float32, device=device)
        self.offsets = torch.zeros(batch + 1, dtype=torch.int32, device=device)

    def pack(self, packer=None, stream=None):
        """Packs the records on the device: ``packer`` is the library's ngsPackResults (on
        ``stream``), or None for pack_torch. The total goes to buf[1]."""
        if packer is None:
            pack_torch(self.counts, self.keys, self.scores, self.batch, self.stride, self.offsets, self.records)
        else:
            rc = packer(self.counts.data_ptr(), self.keys.data_ptr(), self.scores.data_ptr(), self.batch,
                        self.stride, self.offsets.data_ptr(), self.records.data_ptr(), stream)
            if rc:
                raise RuntimeError(f"ngsPackResults -> {rc}")
        self.buf[1:2].copy_(self.offsets[self.batch:self.batch + 1])
        return self

    @staticmethod
    def words(pad_b: int, total: int) -> int:
        """int32 words of a packed buffer holding `total` records."""
        return 2 + pad_b + 2 * total

    @staticmethod
    def decode(buf: torch.Tensor, pad_b: int):
        """(counts, keys, scores) of a gathered packed buffer (its first words(pad_b, cap) words)."""
        b, t = int(buf[0]), int(buf[1])
        if not 0 <= b <= pad_b or buf.numel() < PackedGather.words(pad_b, t):
            raise ValueError(f"gathered buffer of batch {b}, {t} records in {buf.numel()} words does not match "
                             f"pad_b {pad_b}")
        counts = buf[2:2 + b]
        rec = buf[2 + pad_b:2 + pad_b + 2 * t].view(t, 2)
        if int(counts.sum()) != t:
            raise ValueError(f"gathered counts sum to {int(counts.sum())}, not the buffer's {t} records")
        return counts, rec[:, 0].contiguous(), rec[:, 1].contiguous().view(torch.float32)


class GatherCap:
    """The record capacity (per rank) of the packed gathers: a number every rank holds without
    exchanging it, because it only changes in PendingPacked.complete(), which every rank calls for
    the same gather at the same step. It starts at a quarter of the fixed layout (``initial``
    overrides) and grows past any overflowing total by an eighth."""

    def __init__(self, pad_b: int, stride: int, initial: int | None = None):
        self.limit = max(1, pad_b * stride)
        self.total = min(self.limit, max(1, initial if initial is not None else self.limit // 4))
        self.regathers = 0

    def observe(self, total: int) -> bool:
        """The all-reduced largest total of a retired gather; True if it overflowed the capacity."""
        over = total > self.total
        if over:
            self.total = min(self.limit, total + total // 8 + 64)
        return over


class PendingPacked:
    """An in-flight packed gather: ``complete()`` orders the current stream after it, reads the
    batch's all-reduced largest total (copied to the host beside the gather, so the read waits for
    nothing newer) and gathers the buffers again in full if the capacity was too small;
    ``wait()`` returns the per-rank (counts, keys, scores) on rank 0 and None elsewhere."""

    def __init__(self, work, pg: PackedGather, bufs, rank, words, group, cap: GatherCap, tot_work, tot_host,
                 tot_event):
        self.work, self.pg, self.bufs, self.rank, self.words = work, pg, bufs, rank, words
        self.group, self.cap, self.tot_work, self.tot_host, self.tot_event = group, cap, tot_work, tot_host, tot_event
        self.done = False
        self.regathered = False

    def complete(self):
        if self.done:
            return
        self.done = True
        self.work.wait()
        if self.tot_event is not None:
            self.tot_event.synchronize()
        else:
            self.tot_work.wait()
        total = int(self.tot_host[0])
        if total > (self.words - 2 - self.pg.pad_b) // 2:  # some rank's records did not fit: gather them whole
            words = PackedGather.words(self.pg.pad_b, total)
            world = dist.get_world_size(self.group)
            bufs = [torch.empty(words, dtype=torch.int32, device=self.pg.buf.device)
                    for _ in range(world)] if self.rank == 0 else None
            dist.gather(self.pg.buf[:words], bufs, dst=0, group=self.group)
            self.bufs, self.words, self.regathered = bufs, words, True
            self.cap.regathers += 1
        self.cap.observe(total)

    def wait(self):
        self.complete()
        if self.rank != 0:
            return None
        return [PackedGather.decode(b, self.pg.pad_b) for b in self.bufs]


def gather_packed(pg: PackedGather, group=None, async_op: bool = False, cap: GatherCap | None = None):
    """Gathers every rank's packed buffer (already packed) on rank 0: the prefix of
    ``cap.total`` records (a quarter of the fixed layout without a cap), plus an 8-byte all-reduce of the
    largest total that PendingPacked.complete() checks. No host read of this batch. Bytes per rank:
    4 * (2 + pad_b + 2 * cap.total)."""
    cap = cap or GatherCap(pg.pad_b, pg.stride)
    tot = pg.buf[1:2].to(torch.int64)
    tot_work = dist.all_reduce(tot, op=dist.ReduceOp.MAX, group=group, async_op=True)
    tot_host, tot_event = tot, None
    if tot.is_cuda:  # the total to pinned host memory on a side stream, ordered after the all-reduce
        side = _side_stream(tot.device)
        side.wait_stream(torch.cuda.current_stream(tot.device))
        with torch.cuda.stream(side):
            tot_work.wait()
            tot_host = torch.empty(1, dtype=torch.int64, pin_memory=True)
            tot_host.copy_(tot, non_blocking=True)
            tot_event = torch.cuda.Event()
            tot_event.record(side)
        tot.record_stream(side)
    words = PackedGather.words(pg.pad_b, cap.total)
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    send = pg.buf[:words]
    bufs = [torch.empty(words, dtype=torch.int32, device=pg.buf.device) for _ in range(world)] if rank == 0 else None
    work = dist.gather(send, bufs, dst=0, group=group, async_op=True)
    pending = PendingPacked(work, pg, bufs, rank, words, group, cap, tot_work, tot_host, tot_event)
    return pending if async_op else pending.wait()


_SIDE = {}


def _side_stream(device):
    if device not in _SIDE:
        _SIDE[device] = torch.cuda.Stream(device)
    return _SIDE[device]
