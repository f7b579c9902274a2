"""Query-batch sharding across GPUs.

Each rank (one process per GPU) holds a replica of the index and scores a contiguous slice
of the batch; the only collective is the gather of the compacted top-k records to rank 0
(RCCL over xGMI with the ``nccl`` backend; ``gloo`` in the CPU tests). Queries share no
state, so nothing else crosses ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(rank: int, world: int, n: int) -> tuple[int, int]:
    """Contiguous slice [lo, hi) of n queries for `rank`."""
    return n * rank // world, n * (rank + 1) // world


def compact(counts: torch.Tensor, keys: torch.Tensor, scores: torch.Tensor, stride: int):
    """(counts[B], keys[B*stride], scores[B*stride]) -> counts, packed keys, packed scores."""
    B = counts.numel()
    mask = torch.arange(stride, device=counts.device).unsqueeze(0) < counts.view(B, 1).to(torch.int64)
    return counts, keys.view(B, stride)[mask], scores.view(B, stride)[mask]


class PendingGather:
    """An in-flight gather (``gather_to_root(..., async_op=True)``): ``wait()`` returns what the
    blocking call returns (the per-rank lists on rank 0, None elsewhere)."""

    def __init__(self, work, buf, bufs, o, pad_k, rank):
        self.work, self.buf, self.bufs, self.o, self.pad_k, self.rank = work, buf, bufs, o, pad_k, rank

    def complete(self):
        """Orders the current stream after the gather (no host synchronisation, no decode)."""
        self.work.wait()

    def wait(self):
        self.work.wait()
        if self.rank != 0:
            return None
        out = []
        o, pad_k = self.o, self.pad_k
        for b in self.bufs:
            nk, nb = int(b[0]), int(b[1])
            out.append((b[2:2 + nb], b[o:o + nk], b[o + pad_k:o + pad_k + nk].view(torch.float32)))
        return out


def gather_to_root(counts: torch.Tensor, pkeys: torch.Tensor, pscores: torch.Tensor, group=None,
                   async_op: bool = False):
    """Gathers every rank's (counts, packed keys, packed scores) on rank 0.

    Two collectives: an all-reduce of the packed length (so every rank pads to the same
    size) and one gather of a single fused buffer per rank. Returns the per-rank lists on
    rank 0 and None elsewhere; with ``async_op`` the gather stays in flight (RCCL runs it on
    its own stream, beside the next batch's kernels) and a PendingGather is returned."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = counts.device
    n = torch.tensor([pkeys.numel(), counts.numel()], dtype=torch.int64, device=dev)
    mx = n.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    pad_k, pad_b = int(mx[0]), int(mx[1])
    buf = torch.zeros(2 + pad_b + 2 * pad_k, dtype=torch.int32, device=dev)
    buf[0] = n[0].to(torch.int32)
    buf[1] = n[1].to(torch.int32)
    buf[2:2 + counts.numel()] = counts.to(torch.int32)
    o = 2 + pad_b
    buf[o:o + pkeys.numel()] = pkeys.to(torch.int32)
    buf[o + pad_k:o + pad_k + pscores.numel()] = pscores.contiguous().view(torch.int32)
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    work = dist.gather(buf, bufs, dst=0, group=group, async_op=True)
    pending = PendingGather(work, buf, bufs, o, pad_k, rank)
    return pending if async_op else pending.wait()
