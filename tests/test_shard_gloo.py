"""CPU: the multi-GPU row sharding + all-gather assembly (shadow_amd/shard.py) with
world_size 2 on the gloo backend.  Each rank produces its row block with the oracle (a
stand-in for the engine, which needs a GPU) and the assembled matrices must equal the
oracle's full matrix -- i.e. sharding, padding and gather order are exact."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from shadow_amd import shard


def test_shard_rows_cover_exactly():
    for A in (0, 1, 7, 64, 1000, 1001):
        for W in (1, 2, 3, 4, 8):
            covered = []
            pers = set()
            for r in range(W):
                r0, r1, per = shard.shard_rows(A, W, r)
                assert 0 <= r0 <= r1 <= A and r1 - r0 <= per
                covered.extend(range(r0, r1))
                pers.add(per)
            assert covered == list(range(A)) and len(pers) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, A_sel, q):
    import torch.distributed as dist

    from oracle import oracle as O
    from shadow_amd import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.random_sparse(V=150, avg_deg=4, seed=77, A=A_sel)
    og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss)
    flags = og.flags()
    A = len(g.attached)

    def block(r0, r1, bufs):
        lat, rel, hops, kind, _ = og.pair_rows(flags, g.attached, r0, r1)
        bufs[0].copy_(torch.from_numpy(lat))
        bufs[1].copy_(torch.from_numpy(rel))
        bufs[2].copy_(torch.from_numpy(hops.astype(np.int32)))

    lat, rel, hops = shard.assemble(dist, block, A, world, rank, "cpu", (torch.float64, torch.float64, torch.int32))
    if rank == 0:
        full = og.pair_rows(flags, g.attached)
        q.put((np.array_equal(lat.numpy().view(np.uint64), full[0].view(np.uint64)),
               np.array_equal(rel.numpy().view(np.uint64), full[1].view(np.uint64)),
               np.array_equal(hops.numpy(), full[2].astype(np.int32))))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("A_sel", [40, 37])  # even and uneven shards
def test_two_rank_gloo_assembly(A_sel):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, A_sel, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert q.get(timeout=10) == (True, True, True)


def _worker_packed(rank, world, port, A_sel, chunks, q):
    """bench.py's exchange: packed [lat | rel | hops] chunk buffers, one all-gather each"""
    import torch.distributed as dist

    from oracle import oracle as O
    from shadow_amd import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.random_sparse(V=150, avg_deg=4, seed=78, A=A_sel)
    og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss)
    flags = og.flags()
    A = len(g.attached)
    r0, r1, per = shard.shard_rows(A, world, rank)
    bounds = shard.chunk_rows(per, chunks)
    full = og.pair_rows(flags, g.attached)
    ok = True
    for c0, n in bounds:
        buf = torch.zeros(shard.packed_bytes(n, A), dtype=torch.uint8)
        lat, rel, hops = shard.pack_views(buf, n, A)
        a, z = r0 + c0, min(r1, r0 + c0 + n)
        if z > a:
            l, r, h, _, _ = og.pair_rows(flags, g.attached, a, z)
            lat[:z - a] = torch.from_numpy(l)
            rel[:z - a] = torch.from_numpy(r)
            hops[:z - a] = torch.from_numpy(h.astype(np.int32))
        gathered = torch.empty(world * buf.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(gathered, buf)
        for rr, (gl, gr, gh) in enumerate(shard.unpack_gathered(gathered, world, n, A)):
            s0, s1, _ = shard.shard_rows(A, world, rr)
            a, z = s0 + c0, min(s1, s0 + c0 + n)
            if z > a:
                ok &= np.array_equal(gl[:z - a].numpy().view(np.uint64), full[0][a:z].view(np.uint64))
                ok &= np.array_equal(gr[:z - a].numpy().view(np.uint64), full[1][a:z].view(np.uint64))
                ok &= np.array_equal(gh[:z - a].numpy(), full[2][a:z].astype(np.int32))
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("A_sel,chunks", [(150, 2), (131, 3)])
def test_two_rank_packed_chunked_exchange(A_sel, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_packed, args=(r, 2, port, A_sel, chunks, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res == [(0, True), (1, True)]


def test_chunk_rows_cover_exactly():
    for per in (0, 1, 63, 64, 500, 1000, 1001):
        for chunks in (1, 2, 3, 4, 8):
            b = shard.chunk_rows(per, chunks)
            assert sum(n for _, n in b) == per
            assert all(o % 64 == 0 for o, _ in b)
            assert [o for o, _ in b] == sorted(o for o, _ in b)


def _worker_exchange(rank, world, port, A_sel, chunks, q):
    """bench.py's own step (shard.RowExchange), run twice, with the oracle as the compute
    stand-in (the engine needs a GPU; tests/test_engine_gpu.py drives the same class with
    the engine's device rows)"""
    import torch.distributed as dist

    from oracle import oracle as O
    from shadow_amd import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.random_sparse(V=160, avg_deg=4, seed=79, A=A_sel)
    og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss)
    flags = og.flags()
    A = len(g.attached)
    ex = shard.RowExchange(dist, A, world, rank, "cpu", chunks)
    calls = []

    def compute(a, z, lat, rel, hops):
        l, r, h, _, _ = og.pair_rows(flags, g.attached, a, z)
        lat[:z - a] = torch.from_numpy(l)
        rel[:z - a] = torch.from_numpy(r)
        hops[:z - a] = torch.from_numpy(h.astype(np.int32))
        calls.append((a, z))

    full = og.pair_rows(flags, g.attached)
    ok = True
    for _ in range(2):  # buffers are reused step after step
        ex.step(compute)
        lat, rel, hops = ex.full()
        ok &= np.array_equal(lat.numpy().view(np.uint64), full[0].view(np.uint64))
        ok &= np.array_equal(rel.numpy().view(np.uint64), full[1].view(np.uint64))
        ok &= np.array_equal(hops.numpy(), full[2].astype(np.int32))
    mine = sorted(set(calls))
    ok &= sum(z - a for a, z in mine) == ex.rows and all(ex.r0 <= a < z <= ex.r1 for a, z in mine)
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("A_sel,chunks", [(160, 1), (150, 2), (131, 3)])
def test_two_rank_row_exchange_step(A_sel, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_exchange, args=(r, 2, port, A_sel, chunks, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res == [(0, True), (1, True)]


def _worker_bench_sharded(rank, world, port, A_sel, chunks, q, packed=False, hops16=False):
    """bench.py's run_sharded -- the timed step of both the headline line and the north-star
    C4 record at every GPU count (barriers, max-over-ranks timing, all-gather-only leg) --
    with the oracle as the compute stand-in on gloo"""
    import sys

    import torch.distributed as dist

    from oracle import oracle as O
    from shadow_amd import synth
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.random_sparse(V=170, avg_deg=4, seed=81, A=A_sel)
    og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss)
    flags = og.flags()
    A = len(g.attached)
    hooks = []

    def compute(a, z, lat, rel, hops):
        l, r, h, _, _ = og.pair_rows(flags, g.attached, a, z)
        lat[:z - a] = torch.from_numpy(l)
        rel[:z - a] = torch.from_numpy(r)
        hops[:z - a] = torch.from_numpy(h.astype(np.int32))

    codec = hc = None
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if packed:
        from rowcodec_ref import RefRowCodec
        codec = RefRowCodec(g)
    if hops16:  # the sparse exchange: 16-bit hop counts (RefHopCodec stands in for the engine's kernels)
        from rowcodec_ref import RefHopCodec
        hc = RefHopCodec()
    run = bench.run_sharded(dist, world, rank, torch.device("cpu"), A, compute, steps=3, warmup=2, chunks=chunks,
                            on_timed_start=lambda: hooks.append("start"), on_timed_end=lambda: hooks.append("end"),
                            on_first_step=lambda: hooks.append("first"), codec=codec, hops16=hc)
    lat, rel, hops = run["exchange"].full()
    full = og.pair_rows(flags, g.attached)
    ok = np.array_equal(lat.numpy().view(np.uint64), full[0].view(np.uint64))
    ok &= np.array_equal(rel.numpy().view(np.uint64), full[1].view(np.uint64))
    ok &= np.array_equal(hops.numpy(), full[2].astype(np.int32))
    ok &= hooks == ["first", "start", "end"]
    ok &= run["elapsed_s"] > 0 and run["allgather_s"] > 0
    if packed:
        ok &= 0 < run["allgather_bytes"] <= sum(p.numel() for p in run["exchange"].packs) * world * 2
    else:
        ok &= run["allgather_bytes"] == sum(p.numel() for p in run["exchange"].packs) * world
    ok &= run["exchange"].hop_bytes == (2 if hops16 else 4)
    # the N-rank fields the bench line carries (sharded_report): each rank's relax time and
    # rows, the exchange alone and its bytes, the same on every rank
    rep = bench.sharded_report(dist, world, run, 3, relax_ms_per_step=1.0 + rank, rows=run["exchange"].rows)
    ok &= rep["per_rank_relax_ms"] == [1.0 + r for r in range(world)]
    ok &= sum(rep["per_rank_rows"]) == A and rep["per_rank_rows"][rank] == run["exchange"].rows
    ok &= rep["step_includes_exchange"] and rep["exchange_ms"] > 0
    ok &= rep["exchange_ms"] == run["allgather_s"] / 3 * 1e3 and rep["allgather_bytes"] == run["allgather_bytes"]
    # the reported time is the max over ranks: every rank holds the same number
    t = torch.tensor([run["elapsed_s"]], dtype=torch.float64)
    tl = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(tl, t)
    ok &= all(float(x) == run["elapsed_s"] for x in tl)
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("A_sel,chunks,packed,hops16", [(170, 1, False, False), (149, 2, False, False),
                                                        (150, 1, True, False), (149, 2, False, True)])
def test_two_rank_bench_run_sharded(A_sel, chunks, packed, hops16):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_bench_sharded, args=(r, 2, port, A_sel, chunks, q, packed, hops16))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res == [(0, True), (1, True)]


def _worker_exchange_packed(rank, world, port, A_sel, chunks, q):
    """RowExchange with a row codec (the engine's payload format, CPU reference codec):
    sizes agreed, payloads all-gathered, every rank's rows unpacked -- the same matrices as
    the oracle's, with fewer bytes than the raw rows"""
    import sys

    import torch.distributed as dist

    from oracle import oracle as O
    from shadow_amd import synth
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from rowcodec_ref import RefRowCodec
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.geometric_complete_ish(V=220, A=A_sel, drop=0.1)
    og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss)
    flags = og.flags()
    A = len(g.attached)
    ex = shard.RowExchange(dist, A, world, rank, "cpu", chunks, codec=RefRowCodec(g))

    def compute(a, z, lat, rel, hops):
        l, r, h, _, _ = og.pair_rows(flags, g.attached, a, z)
        lat[:z - a] = torch.from_numpy(l)
        rel[:z - a] = torch.from_numpy(r)
        hops[:z - a] = torch.from_numpy(h.astype(np.int32))

    full = og.pair_rows(flags, g.attached)
    ok = True
    for _ in range(2):
        ex.step(compute)
        lat, rel, hops = ex.full()
        ok &= np.array_equal(lat.numpy().view(np.uint64), full[0].view(np.uint64))
        ok &= np.array_equal(rel.numpy().view(np.uint64), full[1].view(np.uint64))
        ok &= np.array_equal(hops.numpy(), full[2].astype(np.int32))
    raw = 2 * sum(p.numel() for p in ex.packs)
    q.put((rank, bool(ok), ex.exchanged_bytes, raw))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("A_sel,chunks", [(120, 1), (131, 2), (65, 1)])
def test_two_rank_packed_row_exchange(A_sel, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_exchange_packed, args=(r, 2, port, A_sel, chunks, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert [(r, ok) for r, ok, _, _ in res] == [(0, True), (1, True)]
    for _, _, sent, raw in res:
        assert sent * 4 < raw, (sent, raw)  # most pairs are the single arc: rebuilt, not sent


def _worker_hops16(rank, world, port, A_sel, chunks, big, q):
    """shard.RowExchange with 16-bit hop counts (the sparse exchange, RefHopCodec standing in
    for the engine's kernels): 18 B per pair, every rank's matrices bit-exact after the
    step; `big` adds 2^16 to some hop counts (a path longer than 65 535 arcs), so the high
    halves are all-gathered too and still round-trip"""
    import sys

    import torch.distributed as dist

    from oracle import oracle as O
    from shadow_amd import synth
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from rowcodec_ref import RefHopCodec
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.random_sparse(V=160, avg_deg=4, seed=83, A=A_sel)
    og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss)
    flags = og.flags()
    A = len(g.attached)
    full = list(og.pair_rows(flags, g.attached))
    want_h = full[2].astype(np.int64)
    if big:
        want_h[::7, ::3] += (1 << 16) + 5  # only in the rows of some ranks' chunks
    ex = shard.RowExchange(dist, A, world, rank, "cpu", chunks, hops16=RefHopCodec())
    ok = ex.hop_bytes == 2
    ok &= all(p.numel() == shard.packed_bytes(n, A, 2) for p, (_, n) in zip(ex.packs, ex.bounds))

    def compute(a, z, lat, rel, hops):
        l, r, _, _, _ = og.pair_rows(flags, g.attached, a, z)
        lat[:z - a] = torch.from_numpy(l)
        rel[:z - a] = torch.from_numpy(r)
        hops[:z - a] = torch.from_numpy(want_h[a:z].astype(np.uint32).view(np.int32))

    for _ in range(2):
        ex.step(compute)
        lat, rel, hops = ex.full()
        ok &= np.array_equal(lat.numpy().view(np.uint64), full[0].view(np.uint64))
        ok &= np.array_equal(rel.numpy().view(np.uint64), full[1].view(np.uint64))
        ok &= np.array_equal(hops.numpy().view(np.uint32).astype(np.int64), want_h)
    ok &= ex.overflowed == (2 * len(ex.bounds) if big else 0)
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("A_sel,chunks,big", [(160, 1, False), (131, 2, False), (150, 2, True)])
def test_two_rank_hops16_exchange(A_sel, chunks, big):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_hops16, args=(r, 2, port, A_sel, chunks, big, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res == [(0, True), (1, True)]


def test_hops16_packed_bytes():
    """18 B per pair (+ the overflow word, 256-byte padded) against 20 B raw; f64 views aligned"""
    for rows, A in ((1, 1), (63, 157), (1250, 10_000)):
        raw, h16 = shard.packed_bytes(rows, A), shard.packed_bytes(rows, A, 2)
        assert h16 % 256 == 0 and h16 >= rows * A * 18 + 8 and h16 <= rows * A * 18 + 8 + 256 + 8
        assert rows * A < 100 or h16 < raw
    buf = torch.zeros(shard.packed_bytes(3, 5, 2), dtype=torch.uint8)
    lat, rel, lo, ovf = shard.pack_views(buf, 3, 5, 2)
    assert lat.shape == (3, 5) and rel.shape == (3, 5) and lo.dtype == torch.int16 and ovf.numel() == 2
