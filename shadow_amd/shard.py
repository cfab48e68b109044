"""Multi-GPU layout of the attached-pair computation.

Sources (attached vertices) are independent, so rank r of W computes the contiguous row
block ``shard_rows(A, W, r)`` of the A x A latency / reliability / hop matrices against
all A targets on its own GPU (the graph is replicated per GPU), and one all-gather per
matrix -- RCCL over xGMI with backend "nccl" -- leaves every rank with the full matrix,
so every host-side lookup is a local table read.  There is no other exchange.

All-gather needs equal-size contributions: every rank contributes ``per = ceil(A/W)``
rows; the last rank's unused rows are padding that ``assemble`` drops.
"""
from __future__ import annotations

import math


def shard_rows(A: int, world: int, rank: int):
    """(row_begin, row_end, per): rank's contiguous block of source rows"""
    per = max(1, math.ceil(A / world)) if A else 0
    r0 = min(A, rank * per)
    r1 = min(A, r0 + per)
    return r0, r1, per


def gather_rows(dist, local, per, world):
    """all_gather of a [per, A] row block -> [world*per, A] (torch tensors, same device)"""
    import torch
    full = torch.empty((per * world,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(full, local.contiguous())
    return full


def assemble(dist, compute_block, A, world, rank, device, dtypes):
    """Run compute_block(r0, r1, buffers) for this rank's rows into zero-padded [per, A]
    buffers (one per dtype), exchange them, return the full [A, A] matrices."""
    import torch
    r0, r1, per = shard_rows(A, world, rank)
    bufs = [torch.zeros((per, A), dtype=dt, device=device) for dt in dtypes]
    if r1 > r0:
        compute_block(r0, r1, [b[:r1 - r0] for b in bufs])
    if world == 1:
        return [b[:A] for b in bufs]
    return [gather_rows(dist, b, per, world)[:A] for b in bufs]
