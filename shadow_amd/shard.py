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


def packed_bytes(rows: int, A: int, hop_bytes: int = 4) -> int:
    """one chunk's lat (f64) + rel (f64) + hops (i32, or with hop_bytes 2 their low 16 bits and
    an 8-byte overflow word) rows in one buffer, padded to a multiple of 256 bytes: rank r's part
    of the all-gathered buffer starts at r * packed_bytes, and its f64 views need 8-byte
    alignment (rows * A odd would otherwise leave ranks >= 1 at an offset of 4 mod 8)"""
    n = rows * A
    if hop_bytes == 2:
        return -(-(16 * n + (2 * n + 7) // 8 * 8 + 8) // 256) * 256
    return -(-n * 20 // 256) * 256


def pack_views(buf, rows: int, A: int, hop_bytes: int = 4):
    """(lat, rel, hops) views [rows, A] into a packed uint8 buffer of packed_bytes(rows, A,
    hop_bytes); with hop_bytes 2 the hops view is int16 (the low halves) and a fourth view is
    the chunk's overflow word (int32[2])"""
    import torch
    n = rows * A
    lat = buf[: 8 * n].view(torch.float64).view(rows, A)
    rel = buf[8 * n: 16 * n].view(torch.float64).view(rows, A)
    if hop_bytes == 2:
        lo = buf[16 * n: 18 * n].view(torch.int16).view(rows, A)
        o = 16 * n + (2 * n + 7) // 8 * 8
        return lat, rel, lo, buf[o: o + 8].view(torch.int32)
    hops = buf[16 * n: 20 * n].view(torch.int32).view(rows, A)
    return lat, rel, hops


def unpack_gathered(gathered, world: int, rows: int, A: int, hop_bytes: int = 4):
    """the all-gathered packed buffer of one chunk -> per-rank (lat, rel, hops[, overflow]) views"""
    per_rank = packed_bytes(rows, A, hop_bytes)
    return [pack_views(gathered[r * per_rank:(r + 1) * per_rank], rows, A, hop_bytes) for r in range(world)]


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


class EngineRowCodec:
    """The row exchange codec of a dense engine (shadowtopo_pack_rows / unpack_rows): a
    rank's rows leave as a payload of one bit per pair that every rank rebuilds from its own
    graph replica (the single arc from the source) plus the other pairs in full; C2 at 8
    ranks moves ~11 MB per rank instead of 160 MB.  Rows are the packed_views of a chunk."""

    def __init__(self, eng, stream_of=None):
        """`stream_of()` -> the hipStream_t the codec's kernels run on.  The default is torch's
        current stream on the engine's device: the payload all-gather and the row buffers are
        ordered on that stream, so packing and unpacking must be too (the engine's own stream
        would let unpack read a payload before the collective has written it)."""
        self.eng = eng
        if stream_of is None:
            import torch
            dev = torch.device("cuda", eng.device)
            stream_of = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731
        self.stream_of = stream_of

    def capacity(self, rows: int, A: int) -> int:
        return self.eng.packed_capacity(rows, A)

    def pack(self, a, z, lat, rel, hops, out) -> int:
        return self.eng.pack_rows(a, z, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), out.data_ptr(), out.numel(),
                                  stream=self.stream_of())

    def unpack(self, a, z, payload, lat, rel, hops):
        self.eng.unpack_rows(a, z, payload.data_ptr(), lat.data_ptr(), rel.data_ptr(), hops.data_ptr(),
                             stream=self.stream_of())


class EngineHopCodec:
    """The sparse row exchange's hop narrowing (shadowtopo_hops_narrow / _widen): hop counts
    travel as their low 16 bits, 18 B per pair instead of 20; a count >= 2^16 sets the chunk's
    overflow word and the high halves follow in a second all-gather.  Runs on torch's current
    stream of the engine's device, the one the collectives are ordered on."""

    def __init__(self, eng, stream_of=None):
        self.eng = eng
        if stream_of is None:
            import torch
            dev = torch.device("cuda", eng.device)
            stream_of = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731
        self.stream_of = stream_of

    def narrow(self, hops, lo, hi, overflow):
        self.eng.hops_narrow(hops.data_ptr(), hops.numel(), lo.data_ptr(), hi.data_ptr() if hi is not None else None,
                             overflow.data_ptr(), stream=self.stream_of())

    def widen(self, lo, hi, out):
        self.eng.hops_widen(lo.data_ptr(), hi.data_ptr() if hi is not None else None, lo.numel(), out.data_ptr(),
                            stream=self.stream_of())


class RowExchange:
    """The multi-GPU step of bench.py: this rank's source rows, computed in
    row chunks of whole 64-source batches into packed [lat | rel | hops] buffers (one
    buffer per chunk, ``pack_views``), each chunk all-gathered asynchronously (RCCL over
    xGMI with backend "nccl") while the next chunk is computed; after ``step`` every rank
    holds every rank's rows.  ``compute(a, z, lat, rel, hops)`` fills rows [a, z) of the
    attached-pair matrix into the [z - a, A] views (the engine on a GPU; tests pass a CPU
    stand-in and the gloo backend)."""

    def __init__(self, dist, A: int, world: int, rank: int, device, chunks: int = 1, codec=None, hops16=None):
        import torch
        self.dist, self.A, self.world, self.rank = dist, A, world, rank
        self.r0, self.r1, self.per = shard_rows(A, world, rank)
        self.bounds = chunk_rows(self.per, chunks)
        # hops16 (a hop codec: EngineHopCodec, or a CPU stand-in in the tests; world > 1, no row
        # codec): the chunks travel with 16-bit hop counts; compute writes its u32 counts into a
        # scratch the codec narrows, and every rank widens the gathered counts into one matrix
        self.hops16 = hops16 if world > 1 and codec is None else None
        hb = 2 if self.hops16 is not None else 4
        self.hop_bytes = hb
        self.packs = [torch.zeros(packed_bytes(n, A, hb), dtype=torch.uint8, device=device) for _, n in self.bounds]
        self.views = [pack_views(b, n, A, hb) for b, (_, n) in zip(self.packs, self.bounds)]
        self.gathered = ([torch.empty(world * p.numel(), dtype=torch.uint8, device=device) for p in self.packs]
                         if world > 1 else None)
        self.overflowed = 0  # steps whose hop counts needed the high halves too (hops16)
        if self.hops16 is not None:
            self.hops32 = [torch.zeros((n, A), dtype=torch.int32, device=device) for _, n in self.bounds]
            self.hi = [torch.zeros((n, A), dtype=torch.int16, device=device) for _, n in self.bounds]
            self.hops_full = torch.zeros((A, A), dtype=torch.int32, device=device)
        # with a codec (world > 1): each chunk leaves as a payload; its size is agreed first
        # (all ranks gather the largest), then the payloads are all-gathered and every rank
        # unpacks every rank's rows into `gathered`, so full() reads the same buffers
        self.codec = codec if world > 1 else None
        self.exchanged_bytes = 0  # payload bytes one rank contributed over the steps (codec)
        if self.codec is not None:
            self.payloads = [torch.empty(codec.capacity(n, A), dtype=torch.uint8, device=device) for _, n in self.bounds]
            # the gathered payloads are sized from the agreed payload size (grown on demand):
            # a packed C2 chunk is ~1/15 of its worst-case capacity
            self.gpay = [torch.empty(0, dtype=torch.uint8, device=device) for _ in self.payloads]
            self.size_t = torch.zeros(1, dtype=torch.int64, device=device)
            self.sizes = torch.zeros(world, dtype=torch.int64, device=device)

    @property
    def rows(self) -> int:
        return self.r1 - self.r0

    def step(self, compute):
        works = []
        for c, (c0, n) in enumerate(self.bounds):
            a, z = self.r0 + c0, min(self.r1, self.r0 + c0 + n)  # this chunk's real rows
            if self.hops16 is not None:
                lat, rel, lo, ovf = self.views[c]
                ovf.zero_()
                if z > a:
                    compute(a, z, lat, rel, self.hops32[c])
                    self.hops16.narrow(self.hops32[c][:z - a], lo[:z - a], self.hi[c][:z - a], ovf)
            elif z > a:
                lat, rel, hops = self.views[c]
                compute(a, z, lat, rel, hops)
            if self.codec is not None:
                self._exchange_packed(c, c0, n, a, z)
            elif self.world > 1:  # returns once the chunk is computed; the gather runs behind the next chunk
                works.append(self.dist.all_gather_into_tensor(self.gathered[c], self.packs[c], async_op=True))
        for w in works:
            w.wait()
        if self.hops16 is not None:
            self._widen_hops()

    def _widen_hops(self):
        """every rank's gathered 16-bit hop counts -> hops_full; the high halves are all-gathered
        first when any rank's chunk overflowed (one flag read per step)"""
        import torch
        parts = [unpack_gathered(self.gathered[c], self.world, n, self.A, 2) for c, (_, n) in enumerate(self.bounds)]
        flags = torch.stack([p[3][0] for pc in parts for p in pc])
        over = bool(flags.any().item())
        for c, (c0, n) in enumerate(self.bounds):
            his = None
            if over:
                self.overflowed += 1
                # as bytes (gloo has no 16-bit integer collectives)
                g = torch.empty(self.world * n * self.A * 2, dtype=torch.uint8, device=self.hi[c].device)
                self.dist.all_gather_into_tensor(g, self.hi[c].view(-1).view(torch.uint8))
                g = g.view(torch.int16).view(self.world * n, self.A)
                his = [g[r * n:(r + 1) * n] for r in range(self.world)]
            for rr in range(self.world):
                s0, s1, _ = shard_rows(self.A, self.world, rr)
                ra, rz = s0 + c0, min(s1, s0 + c0 + n)
                if rz > ra:
                    self.hops16.widen(parts[c][rr][2][:rz - ra], his[rr][:rz - ra] if his else None,
                                      self.hops_full[ra:rz])

    def _exchange_packed(self, c, c0, n, a, z):
        lat, rel, hops = self.views[c]
        nbytes = self.codec.pack(a, z, lat[:z - a], rel[:z - a], hops[:z - a], self.payloads[c]) if z > a else 0
        self.size_t.fill_(nbytes)
        self.dist.all_gather_into_tensor(self.sizes, self.size_t)
        m = max(256, int(self.sizes.max().item()))  # every rank's slot in the gathered payloads
        if self.gpay[c].numel() < self.world * m:
            import torch
            self.gpay[c] = torch.empty(self.world * m, dtype=torch.uint8, device=self.payloads[c].device)
        self.exchanged_bytes += m
        self.dist.all_gather_into_tensor(self.gpay[c][:self.world * m], self.payloads[c][:m])
        parts = unpack_gathered(self.gathered[c], self.world, n, self.A)
        for rr in range(self.world):
            s0, s1, _ = shard_rows(self.A, self.world, rr)
            ra, rz = s0 + c0, min(s1, s0 + c0 + n)
            if rz > ra:
                pl, pr, ph = parts[rr]
                self.codec.unpack(ra, rz, self.gpay[c][rr * m:(rr + 1) * m], pl[:rz - ra], pr[:rz - ra], ph[:rz - ra])

    def full(self):
        """the assembled [A, A] lat, rel, hops (torch, on the buffers' device) after step()"""
        import torch
        dev = self.packs[0].device
        out = (torch.empty((self.A, self.A), dtype=torch.float64, device=dev),
               torch.empty((self.A, self.A), dtype=torch.float64, device=dev),
               torch.empty((self.A, self.A), dtype=torch.int32, device=dev))
        for c, (c0, n) in enumerate(self.bounds):
            parts = (unpack_gathered(self.gathered[c], self.world, n, self.A, self.hop_bytes) if self.world > 1
                     else [self.views[c]])
            for rr, views in enumerate(parts):
                s0, s1, _ = shard_rows(self.A, self.world, rr)
                a, z = s0 + c0, min(s1, s0 + c0 + n)
                if z > a:
                    for o, v in zip(out[:2], views[:2]):
                        o[a:z] = v[:z - a]
                    out[2][a:z] = self.hops_full[a:z] if self.hops16 is not None else views[2][:z - a]
        return out
