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


def chunk_rows(per: int, chunks: int):
    """[(offset, rows)] splitting a rank's `per` rows into `chunks` pieces of whole 64-source
    batches (the last may be short); the same split on every rank, so chunk c's buffers have
    one size everywhere (all-gather needs equal contributions)"""
    chunks = max(1, chunks)
    n = max(64, -(-per // chunks // 64) * 64) if per else 0
    out, o = [], 0
    while o < per:
        out.append((o, min(n, per - o)))
        o += n
    return out or [(0, 0)]


def packed_bytes(rows: int, A: int) -> int:
    """one chunk's lat (f64) + rel (f64) + hops (i32) rows in one buffer"""
    return rows * A * 20


def pack_views(buf, rows: int, A: int):
    """(lat, rel, hops) views [rows, A] into a packed uint8 buffer of packed_bytes(rows, A)"""
    import torch
    n = rows * A
    lat = buf[: 8 * n].view(torch.float64).view(rows, A)
    rel = buf[8 * n: 16 * n].view(torch.float64).view(rows, A)
    hops = buf[16 * n: 20 * n].view(torch.int32).view(rows, A)
    return lat, rel, hops


def unpack_gathered(gathered, world: int, rows: int, A: int):
    """the all-gathered packed buffer of one chunk -> per-rank (lat, rel, hops) views"""
    per_rank = packed_bytes(rows, A)
    return [pack_views(gathered[r * per_rank:(r + 1) * per_rank], rows, A) for r in range(world)]


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
