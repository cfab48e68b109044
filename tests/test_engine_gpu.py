"""GPU parity: libshadowtopo_hip (through its C ABI) against the CPU oracle.

Bar: latency, hop count, pair kind and reliability bit-exact (the engine folds in the
reference's order, topology.c:1429-1499); the north-star tolerance for reliability is
1e-9 relative, which bit-exactness satisfies.
"""
import numpy as np
import pytest

from paritylib import assert_bitexact, compare, engine_matrix, oracle_for, oracle_matrix
from shadow_amd import engine as E
from shadow_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_sparse_undirected(seed):
    g = synth.random_sparse(V=400, avg_deg=5, seed=seed)
    st = compare(g)
    assert st["replayed_sources"] == 0


def test_random_sparse_subset_attached():
    g = synth.random_sparse(V=900, avg_deg=3, seed=7, A=150)
    compare(g)


def test_more_than_one_batch_group():
    g = synth.random_sparse(V=300, avg_deg=4, seed=9)
    # 300 sources -> 5 batches; force 2 batches in flight -> 3 groups
    compare(g, batches_in_flight=2)


def test_directed():
    g = synth.random_sparse(V=300, avg_deg=4, seed=5, directed=True)
    compare(g)


def test_no_self_loops():
    g = synth.random_sparse(V=250, avg_deg=4, seed=4, loops=False)
    compare(g)


@pytest.mark.parametrize("shape", [1, 2])
def test_vertex_loss_walk(shape):
    """targets with vertex loss take k_walk's full fold; both walk shapes (OPT_WALK_TPW)"""
    rng = np.random.default_rng(3)
    vl = np.where(rng.random(300) < 0.5, rng.uniform(0, 0.1, 300), np.nan)
    g = synth.random_sparse(V=300, avg_deg=4, seed=12, vloss=vl)
    compare(g, walk_tpw=shape)


def test_prefer_direct():
    g = synth.random_sparse(V=300, avg_deg=6, seed=13)
    g.prefer_direct = True
    compare(g)


def test_self_dijkstra_loop_rule():
    g = synth.random_sparse(V=200, avg_deg=4, seed=14)
    compare(g, self_loop_rule=True)


def test_integer_ties_replayed():
    g = synth.integer_grid(rows=12, cols=12, seed=3)
    st = compare(g)
    assert st["replayed_sources"] > 0


def test_integer_random_ties():
    g = synth.random_sparse(V=300, avg_deg=5, seed=15, int_lat=True)
    compare(g)


def test_force_replay_matches():
    g = synth.random_sparse(V=200, avg_deg=4, seed=16)
    st = compare(g, force_replay=1)
    assert st["replayed_sources"] == g.attached.size


@pytest.mark.parametrize("shape", [1, 2])
def test_multigraph_parallel_edges(shape):
    g = synth.random_sparse(V=150, avg_deg=4, seed=17)
    # duplicate 40 edges with different latency/loss (parallel edges)
    rng = np.random.default_rng(0)
    pick = rng.choice(np.nonzero(g.src != g.dst)[0], 40, replace=False)
    g.src = np.concatenate([g.src, g.dst[pick]])
    g.dst = np.concatenate([g.dst, g.src[pick]])
    g.latency = np.concatenate([g.latency, g.latency[pick] * rng.uniform(0.3, 1.7, 40)])
    g.packetloss = np.concatenate([g.packetloss, rng.uniform(0, 0.05, 40)])
    compare(g, walk_tpw=shape)


def test_complete_graph_direct_rule():
    n = 40
    iu, ju = np.triu_indices(n, 0)
    rng = np.random.default_rng(2)
    g = synth._finish("complete", n, iu, ju, rng.uniform(1, 50, len(iu)), rng.uniform(0, 0.05, len(iu)),
                      np.arange(n))
    og = oracle_for(g)
    assert og.is_complete()
    compare(g)


def test_geometric_small():
    g = synth.geometric_complete_ish(V=600, A=100)
    compare(g)


def test_sssp_full_rows_vs_oracle():
    g = synth.random_sparse(V=500, avg_deg=4, seed=21)
    og = oracle_for(g)
    eng = E.Engine.from_synth(g)
    srcs = np.array([0, 7, 99, 250, 499], np.int32)
    dist, pred, hops, tie = eng.sssp(srcs)
    for k, s in enumerate(srcs):
        d, parent = og.dijkstra(int(s))
        dd = np.where(d < 0, np.inf, d)
        assert np.array_equal(dist[k].view(np.uint64), dd.view(np.uint64))
        # predecessor vertex from igraph parent edge
        pv = np.where(parent >= 0, np.where(og.src[np.maximum(parent, 0)] == np.arange(g.n),
                                            og.dst[np.maximum(parent, 0)], og.src[np.maximum(parent, 0)]), -1)
        notie = tie[k] == 0
        assert np.array_equal(pred[k][notie], pv[notie])
    eng.close()


# ---- dense-tile relaxation (k_relax_dense): forced on graphs of every shape
@pytest.mark.parametrize("seed", [1, 2])
def test_dense_layout_sparse_graph(seed):
    g = synth.random_sparse(V=301, avg_deg=5, seed=seed)  # odd V: padding row / column
    st = compare(g, layout="dense")
    assert st["dense"] == 1


def test_dense_layout_directed():
    g = synth.random_sparse(V=203, avg_deg=4, seed=5, directed=True)
    assert compare(g, layout="dense")["dense"] == 1


def test_dense_layout_vertex_loss_and_prefer_direct():
    rng = np.random.default_rng(4)
    g = synth.random_sparse(V=150, avg_deg=8, seed=6, vloss=rng.uniform(0, 0.1, 150))
    g.prefer_direct = True
    assert compare(g, layout="dense")["dense"] == 1


def test_dense_layout_ties_and_multigraph():
    g = synth.integer_grid(rows=9, cols=11, seed=2)
    st = compare(g, layout="dense")
    assert st["dense"] == 1 and st["replayed_sources"] > 0
    g = synth.random_sparse(V=100, avg_deg=4, seed=17)
    rng = np.random.default_rng(1)
    pick = rng.choice(np.nonzero(g.src != g.dst)[0], 30, replace=False)
    g.src = np.concatenate([g.src, g.dst[pick]])
    g.dst = np.concatenate([g.dst, g.src[pick]])
    g.latency = np.concatenate([g.latency, g.latency[pick] * rng.uniform(0.3, 1.7, 30)])
    g.packetloss = np.concatenate([g.packetloss, rng.uniform(0, 0.05, 30)])
    compare(g, layout="dense")


def test_geometric_auto_dense():
    g = synth.geometric_complete_ish(V=700, A=130)
    st = compare(g)
    assert st["dense"] == 1  # complete-ish: auto layout picks dense


def test_csr_forced_on_dense_graph():
    g = synth.geometric_complete_ish(V=300, A=70)
    st = compare(g, layout="csr")
    assert st["dense"] == 0


@pytest.mark.parametrize("variant", [E.DENSE_F32, E.DENSE_F64])
def test_dense_variants_agree(variant):
    g = synth.random_sparse(V=333, avg_deg=6, seed=23)
    assert compare(g, layout="dense", dense_variant=variant)["dense"] == 1


# ---- dense delta rounds (k_relax_dense_delta): change-mask rounds after the first sweep
@pytest.mark.parametrize("variant", [E.DENSE_F32, E.DENSE_F64])
@pytest.mark.parametrize("permille", [0, 1000])
@pytest.mark.parametrize("case", ["sparse", "directed", "ties", "vloss_prefer", "multigraph", "geometric"])
def test_dense_delta_rounds(case, permille, variant):
    if case == "sparse":
        g = synth.random_sparse(V=301, avg_deg=5, seed=2)
    elif case == "directed":
        g = synth.random_sparse(V=203, avg_deg=4, seed=5, directed=True)
    elif case == "ties":
        g = synth.integer_grid(rows=9, cols=11, seed=2)
    elif case == "vloss_prefer":
        rng = np.random.default_rng(4)
        g = synth.random_sparse(V=150, avg_deg=8, seed=6, vloss=rng.uniform(0, 0.1, 150))
        g.prefer_direct = True
    elif case == "multigraph":
        g = synth.random_sparse(V=100, avg_deg=4, seed=17)
        rng = np.random.default_rng(1)
        pick = rng.choice(np.nonzero(g.src != g.dst)[0], 30, replace=False)
        g.src = np.concatenate([g.src, g.dst[pick]])
        g.dst = np.concatenate([g.dst, g.src[pick]])
        g.latency = np.concatenate([g.latency, g.latency[pick] * rng.uniform(0.3, 1.7, 30)])
        g.packetloss = np.concatenate([g.packetloss, rng.uniform(0, 0.05, 30)])
    else:
        g = synth.geometric_complete_ish(V=700, A=130)
    st = compare(g, layout="dense", delta_permille=permille, dense_variant=variant)
    assert st["dense"] == 1
    if permille == 0:
        assert st["delta_sweeps"] == 0
    else:
        assert st["delta_sweeps"] > 0 and st["full_sweeps"] == 1  # only the first sweep is full


@pytest.mark.parametrize("case", ["ties", "sparse"])
def test_dense_delta_same_fixed_point(case):
    """Full sweeps and delta rounds must reach the same state: distances bit-exact, tie flags
    identical, predecessor and hops identical wherever no heap-order tie is involved."""
    g = synth.integer_grid(rows=12, cols=13, seed=4) if case == "ties" else synth.random_sparse(V=400, avg_deg=6, seed=8)
    srcs = np.arange(0, g.n, 3, dtype=np.int32)
    outs = []
    for permille, variant in ((0, E.DENSE_F32), (1000, E.DENSE_F32), (1000, E.DENSE_F64), (0, E.DENSE_F64)):
        eng = E.Engine.from_synth(g, layout="dense")
        eng.set_option(E.OPT_DELTA_PERMILLE, permille)
        eng.set_option(E.OPT_DENSE_VARIANT, variant)
        outs.append(eng.sssp(srcs))
        eng.close()
    (d0, p0, h0, t0) = outs[0]
    for d1, p1, h1, t1 in outs[1:]:
        assert np.array_equal(d0.view(np.uint64), d1.view(np.uint64))
        assert np.array_equal(t0, t1)
        ok = t0 == 0
        assert np.array_equal(p0[ok], p1[ok]) and np.array_equal(h0[ok], h1[ok])
    if case == "ties":
        assert (t0 != 0).any()


@pytest.mark.parametrize("case", ["sparse", "directed", "ties", "vloss_prefer", "geometric_odd"])
def test_dense_fused_seed_same_state(case):
    """OPT_DENSE_SEED: the fused round-0 kernel (k_seed_dense_t) and the init / source seed /
    arc seed kernels leave the same state, so rows and matrices are bit-identical (and the
    default, fused, matches the oracle)."""
    if case == "sparse":
        g = synth.random_sparse(V=301, avg_deg=5, seed=2)
    elif case == "directed":
        g = synth.random_sparse(V=203, avg_deg=4, seed=5, directed=True)
    elif case == "ties":
        g = synth.integer_grid(rows=9, cols=11, seed=2)
    elif case == "vloss_prefer":
        rng = np.random.default_rng(4)
        g = synth.random_sparse(V=150, avg_deg=8, seed=6, vloss=rng.uniform(0, 0.1, 150))
        g.prefer_direct = True
    else:
        g = synth.geometric_complete_ish(V=611, A=150)  # V not a multiple of 64, 3 batches
    srcs = np.arange(0, g.n, 2, dtype=np.int32)
    rows, mats = [], []
    for fused in (0, 1):
        eng = E.Engine.from_synth(g, layout="dense")
        eng.set_option(E.OPT_DENSE_SEED, fused)
        rows.append(eng.sssp(srcs))
        eng.set_attached(g.attached)
        mats.append(eng.compute_rows(want_kind=True))
        eng.close()
    (d0, p0, h0, t0), (d1, p1, h1, t1) = rows
    assert np.array_equal(d0.view(np.uint64), d1.view(np.uint64))
    assert np.array_equal(t0, t1)
    ok = t0 == 0
    assert np.array_equal(p0[ok], p1[ok]) and np.array_equal(h0[ok], h1[ok])
    for x, y in zip(*mats):
        assert np.array_equal(x.view(np.uint8) if x.dtype == np.float64 else x,
                              y.view(np.uint8) if y.dtype == np.float64 else y)
    assert compare(g, layout="dense")["dense"] == 1


@pytest.mark.parametrize("case", ["sparse", "directed", "ties", "vloss_prefer", "geometric_odd", "geometric_big"])
def test_dense_prune_same_results(case):
    """OPT_DENSE_PRUNE: the pruned full sweep (vertex locality order, chunks skipped on the
    min-D32 / min-W32 bound, sources batched in locality order) gives bit-identical rows and
    matrices to the unpruned sweep, and the default (pruned) matches the oracle."""
    if case == "sparse":
        g = synth.random_sparse(V=301, avg_deg=5, seed=2)
    elif case == "directed":
        g = synth.random_sparse(V=203, avg_deg=4, seed=5, directed=True)
    elif case == "ties":
        g = synth.integer_grid(rows=9, cols=11, seed=2)
    elif case == "vloss_prefer":
        rng = np.random.default_rng(4)
        g = synth.random_sparse(V=150, avg_deg=8, seed=6, vloss=rng.uniform(0, 0.1, 150))
        g.prefer_direct = True
    elif case == "geometric_odd":
        g = synth.geometric_complete_ish(V=611, A=150)  # V not a multiple of 64, 3 batches
    else:
        g = synth.geometric_complete_ish(V=2500, A=400, drop=0.2)  # 7 batches, many skipped chunks
    srcs = np.arange(0, g.n, 3, dtype=np.int32)
    rows, mats = [], []
    for prune, permille in ((0, 125), (1, 125), (1, 1000)):
        eng = E.Engine.from_synth(g, layout="dense")
        eng.set_option(E.OPT_DENSE_PRUNE, prune)
        eng.set_option(E.OPT_DELTA_PERMILLE, permille)  # 1000: every round after the first is a delta round
        eng.set_attached(g.attached)
        mats.append(eng.compute_rows(want_kind=True))  # builds the vertex order when pruning
        rows.append(eng.sssp(srcs))  # full rows through the (pruned) sweep and delta rounds
        st = eng.stats()
        if prune:  # every delta round in the locality order (chunk bounds) or over live-chunk lists
            assert st["pruned_deltas"] + st["sparse_deltas"] == st["delta_sweeps"]
            if case == "geometric_big":
                assert st["pruned_deltas"] > 0
        eng.close()
    assert np.array_equal(rows[1][0].view(np.uint64), rows[2][0].view(np.uint64))
    for x, y in zip(mats[1], mats[2]):
        assert np.array_equal(x.view(np.uint8) if x.dtype == np.float64 else x,
                              y.view(np.uint8) if y.dtype == np.float64 else y)
    rows, mats = rows[:2], mats[:2]
    (d0, p0, h0, t0), (d1, p1, h1, t1) = rows
    assert np.array_equal(d0.view(np.uint64), d1.view(np.uint64))
    assert np.array_equal(t0, t1)
    ok = t0 == 0
    assert np.array_equal(p0[ok], p1[ok]) and np.array_equal(h0[ok], h1[ok])
    for x, y in zip(*mats):
        assert np.array_equal(x.view(np.uint8) if x.dtype == np.float64 else x,
                              y.view(np.uint8) if y.dtype == np.float64 else y)
    if case != "geometric_big":
        assert compare(g, layout="dense")["dense"] == 1


@pytest.mark.parametrize("layout", ["csr", "dense"])
def test_pinned_host_rows_pipelined(layout):
    """Rows into page-locked host memory (the shim's path): with several batch groups the
    copy of group g runs on the copy stream behind group g + 1 through two staging slots;
    without hops (the shim never copies them).  Bit-identical to pageable buffers and to the
    oracle."""
    g = synth.random_sparse(V=700, avg_deg=5, seed=52, A=500)
    lat_o, rel_o, hops_o, kind_o, _ = oracle_matrix(g)
    eng = E.Engine.from_synth(g, layout=layout)
    eng.set_option(E.OPT_BATCHES_IN_FLIGHT, 2)  # 500 rows -> 8 batches -> 4 groups
    eng.set_attached(g.attached)
    A = len(g.attached)
    lat = E.pinned_empty((A, A), np.float64)
    rel = E.pinned_empty((A, A), np.float64)
    kind = E.pinned_empty((A, A), np.uint8)
    lat[:] = 7.0
    eng.compute_rows_into(0, A, lat, rel, None, kind)
    assert_bitexact("latency", lat, lat_o)
    assert_bitexact("reliability", rel, rel_o)
    assert_bitexact("kind", kind, kind_o)
    # a sub-range with hops, pinned, against the pageable path
    hops = E.pinned_empty((A - 130, A), np.uint32)
    lat2 = E.pinned_empty((A - 130, A), np.float64)
    rel2 = E.pinned_empty((A - 130, A), np.float64)
    eng.compute_rows_into(100, A - 30, lat2, rel2, hops, None)
    pl, pr, ph, _ = eng.compute_rows(100, A - 30, want_kind=False)
    eng.close()
    assert_bitexact("latency", lat2, pl)
    assert_bitexact("reliability", rel2, pr)
    assert_bitexact("hops", hops, ph)
    assert_bitexact("hops", hops, hops_o[100:A - 30])


def test_pinned_host_rows_split_into_groups():
    """A sparse computation that fits one batch group but whose rows pass 64 MB is cut into
    host groups of at least 24 batches (up to opt_host_split = 4), so its copies overlap the
    later groups' rounds: 3200 sources of a k-NN graph (174 MB of rows, 50 batches -> 2
    groups).  Bit-identical to the pageable path, which computes in one group (fewer rounds)."""
    g = synth.knn_geographic(V=3200, k=8, seed=12)
    eng = E.Engine.from_synth(g, layout="csr")
    eng.set_attached(g.attached)
    A = len(g.attached)
    lat = E.pinned_empty((A, A), np.float64)
    rel = E.pinned_empty((A, A), np.float64)
    kind = E.pinned_empty((A, A), np.uint8)
    r0 = eng.stats()["rounds"]
    eng.compute_rows_into(0, A, lat, rel, None, kind)
    r1 = eng.stats()["rounds"]
    pl, pr, _, pk = eng.compute_rows(0, A, want_kind=True)
    r2 = eng.stats()["rounds"]
    eng.close()
    assert r1 - r0 > r2 - r1, (r1 - r0, r2 - r1)
    assert_bitexact("latency", lat, pl)
    assert_bitexact("reliability", rel, pr)
    assert_bitexact("kind", kind, pk)


@pytest.mark.parametrize("layout", ["csr", "dense"])
def test_host_groups_forced(layout):
    """OPT_HOST_GROUPS: rows into page-locked memory in a forced number of batch groups (each
    group's copy behind the next group's rounds), bit-identical to the pageable path"""
    g = synth.random_sparse(V=600, avg_deg=5, seed=53, A=400)
    eng = E.Engine.from_synth(g, layout=layout)
    eng.set_option(E.OPT_HOST_GROUPS, 3)
    eng.set_attached(g.attached)
    A = len(g.attached)
    outs = [E.pinned_empty((A, A), np.float64), E.pinned_empty((A, A), np.float64),
            E.pinned_empty((A, A), np.uint32), E.pinned_empty((A, A), np.uint8)]
    eng.reset_stats()
    eng.compute_rows_into(0, A, *outs)
    assert eng.stats()["groups"] == 3
    want = eng.compute_rows(0, A, want_kind=True)
    eng.close()
    for name, got, w in zip(("latency", "reliability", "hops", "kind"), outs, want):
        assert_bitexact(name, got, w)


def test_row_exchange_with_engine_device_rows():
    """bench.py's step (shard.RowExchange) with the engine's device rows (compute_rows_device
    on torch's stream) in two row chunks, world size 1: the assembled matrix equals the
    oracle's"""
    import torch

    from shadow_amd import shard
    g = synth.random_sparse(V=600, avg_deg=5, seed=53, A=300)
    lat_o, rel_o, hops_o, _, _ = oracle_matrix(g)
    eng = E.Engine.from_synth(g)
    eng.set_attached(g.attached)
    dev = torch.device("cuda:0")
    ex = shard.RowExchange(None, len(g.attached), 1, 0, dev, chunks=2)
    assert len(ex.bounds) == 2

    def compute(a, z, lat, rel, hops):
        eng.compute_rows_device(a, z, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(),
                                stream=torch.cuda.current_stream(dev).cuda_stream)

    ex.step(compute)
    torch.cuda.synchronize(dev)
    lat, rel, hops = (x.cpu().numpy() for x in ex.full())
    eng.close()
    assert_bitexact("latency", lat, lat_o)
    assert_bitexact("reliability", rel, rel_o)
    assert_bitexact("hops", hops.astype(np.uint32), hops_o)


@pytest.mark.parametrize("big", [False, True])
def test_hops16_codec_round_trip(big):
    """shadowtopo_hops_narrow / _widen (shard.EngineHopCodec, the sparse row exchange): u32 hop
    counts -> 16-bit halves and back, bit-exact; the overflow word is set exactly when a count
    reaches 2^16, and widening without the high halves keeps the low ones"""
    import torch

    from shadow_amd import shard
    g = synth.random_sparse(V=300, avg_deg=4, seed=55)
    eng = E.Engine.from_synth(g)
    dev = torch.device("cuda:0")
    codec = shard.EngineHopCodec(eng)
    n = 3 * 65536 + 77  # past one grid-stride pass of the narrowing kernel
    rng = np.random.default_rng(8)
    h = rng.integers(0, 1 << 16 if not big else 1 << 20, n, dtype=np.int64)
    hops = torch.from_numpy(h.astype(np.uint32).view(np.int32)).to(dev)
    lo = torch.empty(n, dtype=torch.int16, device=dev)
    hi = torch.empty(n, dtype=torch.int16, device=dev)
    ovf = torch.zeros(2, dtype=torch.int32, device=dev)
    codec.narrow(hops, lo, hi, ovf)
    back = torch.empty(n, dtype=torch.int32, device=dev)
    codec.widen(lo, hi, back)
    low = torch.empty(n, dtype=torch.int32, device=dev)
    codec.widen(lo, None, low)
    torch.cuda.synchronize(dev)
    eng.close()
    assert int(ovf[0].item()) == (1 if big else 0) and int(ovf[1].item()) == 0
    assert np.array_equal(back.cpu().numpy().view(np.uint32).astype(np.int64), h)
    assert np.array_equal(low.cpu().numpy().view(np.uint32).astype(np.int64), h & 0xFFFF)


def test_row_exchange_hops16_with_engine_device_rows():
    """RowExchange's 16-bit hop path with the engine's device rows and kernels, as rank 0 of
    two with a one-process stand-in of the collective: rank 0's assembled rows equal the
    oracle's (the two-rank exchange itself runs on gloo in tests/test_shard_gloo.py)"""
    import torch

    from shadow_amd import shard

    class OneRank:
        def all_gather_into_tensor(self, out, inp, async_op=False):
            k = out.numel() // inp.numel()
            out.view(k, -1).copy_(inp.reshape(1, -1).expand(k, -1))

            class W:
                def wait(self):
                    pass
            return W() if async_op else None

    g = synth.random_sparse(V=600, avg_deg=5, seed=57, A=300)
    lat_o, rel_o, hops_o, _, _ = oracle_matrix(g)
    eng = E.Engine.from_synth(g)
    eng.set_attached(g.attached)
    dev = torch.device("cuda:0")
    # force the 16-bit path at one rank (the constructor enables it from two ranks on)
    ex2 = shard.RowExchange(OneRank(), len(g.attached), 2, 0, dev, chunks=2, hops16=shard.EngineHopCodec(eng))
    assert ex2.hop_bytes == 2

    def compute(a, z, lat, rel, hops):
        eng.compute_rows_device(a, z, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(),
                                stream=torch.cuda.current_stream(dev).cuda_stream)

    # two ranks' worth of rows computed by this one process: rank 1's half is gathered as a copy
    # of rank 0's buffer, so only rank 0's rows are checked
    ex2.step(compute)
    torch.cuda.synchronize(dev)
    lat, rel, hops = (x.cpu().numpy() for x in ex2.full())
    eng.close()
    r1 = ex2.r1
    assert_bitexact("latency", lat[:r1], lat_o[:r1])
    assert_bitexact("reliability", rel[:r1], rel_o[:r1])
    assert_bitexact("hops", hops[:r1].astype(np.uint32), hops_o[:r1])
    assert ex2.overflowed == 0


@pytest.mark.parametrize("live", ["0", "1"])
@pytest.mark.parametrize("case", ["ties", "geometric", "directed", "vloss_prefer"])
def test_dense_delta_live_chunks(case, live):
    """Delta rounds that walk only the 64-row chunks holding a changed row (k_live_chunks)
    against the full walk: the same matrices, bit for bit, and the oracle's.  Forced on for
    every delta round (OPT_DELTA_LIVE=1) and off (=0)."""
    if case == "ties":
        g = synth.integer_grid(rows=11, cols=12, seed=6)
    elif case == "directed":
        g = synth.random_sparse(V=260, avg_deg=5, seed=9, directed=True)
    elif case == "vloss_prefer":
        rng = np.random.default_rng(5)
        g = synth.random_sparse(V=170, avg_deg=8, seed=7, vloss=rng.uniform(0, 0.1, 170))
        g.prefer_direct = True
    else:
        g = synth.geometric_complete_ish(V=900, A=200)
    # (the live-chunk lists serve the unpruned order; the pruned delta rounds bound chunks
    # themselves: test_dense_prune_same_results)
    st = compare(g, layout="dense", delta_permille=1000, dense_prune=0, delta_live=int(live))
    assert st["dense"] == 1 and st["delta_sweeps"] > 0
    assert (st["sparse_deltas"] > 0) == (live == "1")


@pytest.mark.gpu
def test_prepare_then_create_same_results():
    """An engine created after shadowtopo_prepare adopts the prepared stream and gives the
    same results as one created without it (the preparation only moves runtime work)."""
    g = synth.random_sparse(V=400, avg_deg=5, seed=31)
    E.prepare(0)
    E.prepare(0)  # idempotent while running or ready
    a = E.Engine.from_synth(g)
    st = a.stats()
    assert st["prepare_ms"] >= 0.0 and st["create_prepare_wait_ms"] >= 0.0
    a.set_attached(g.attached)
    ra = a.compute_rows(0, len(g.attached))
    b = E.Engine.from_synth(g)  # no preparation pending: creates its own stream
    b.set_attached(g.attached)
    rb = b.compute_rows(0, len(g.attached))
    for x, y in zip(ra, rb):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("case", ["sparse", "groups", "ties", "vloss_prefer", "multigraph", "pendant", "worklist", "grid"])
def test_push_rounds_same_results(case):
    """SHADOWTOPO_CSR_PUSH (distance pushes with a u64 atomicMin, the exact predecessor pass,
    the fold rounds) against the oracle, bit for bit: several batch groups, integer-latency
    ties (the replay path), vertex loss + prefer-direct, parallel edges, pendant trees, and the
    worklist / grid round forms forced"""
    opts = {}
    if case == "groups":
        g = synth.random_sparse(V=500, avg_deg=4, seed=21)
        opts["batches_in_flight"] = 3
    elif case == "ties":
        g = synth.integer_grid(rows=12, cols=12, seed=3)
    elif case == "vloss_prefer":
        rng = np.random.default_rng(4)
        g = synth.random_sparse(V=200, avg_deg=5, seed=19, vloss=rng.uniform(0, 0.05, 200))
        g.prefer_direct = True
    elif case == "multigraph":
        g = synth.random_sparse(V=150, avg_deg=4, seed=17)
        rng = np.random.default_rng(0)
        pick = rng.choice(np.nonzero(g.src != g.dst)[0], 40, replace=False)
        g.src = np.concatenate([g.src, g.dst[pick]])
        g.dst = np.concatenate([g.dst, g.src[pick]])
        g.latency = np.concatenate([g.latency, g.latency[pick] * rng.uniform(0.3, 1.7, 40)])
        g.packetloss = np.concatenate([g.packetloss, rng.uniform(0, 0.05, 40)])
    elif case == "pendant":
        g = synth.chung_lu(V=3000, A=300, seeds=(7, 8))
    else:
        g = synth.random_sparse(V=600, avg_deg=3, seed=23, A=200)
        opts["worklist"] = 2 if case == "worklist" else 0
    st = compare(g, layout="csr", csr_variant=E.CSR_PUSH, **opts)
    assert st["push_rounds"] > 0 and st["fold_rounds"] > 0
    if case == "ties":
        assert st["replayed_sources"] > 0


def test_push_rounds_rejects_directed():
    g = synth.random_sparse(V=100, avg_deg=4, seed=5, directed=True)
    eng = E.Engine.from_synth(g)
    with pytest.raises(E.ShadowTopoError):
        eng.set_option(E.OPT_CSR_VARIANT, E.CSR_PUSH)
    eng.close()


@pytest.mark.parametrize("case", ["geometric", "geometric_odd", "geometric_huge", "ties", "vloss_prefer"])
def test_dense_w16_filter_same_results(case):
    """OPT_DENSE_W16: the pruned sweep's chunk loop filters with fp16 weights rounded down
    (half the LDS slab and table); the matrices are bit for bit the f32 filter's and the
    oracle's.  The geometric graph has latencies up to ~280 ms (fp16 ulp 0.25 ms there)."""
    if case == "geometric":
        g = synth.geometric_complete_ish(V=2000, A=300)
    elif case == "geometric_odd":
        g = synth.geometric_complete_ish(V=1337, A=257)
    elif case == "geometric_huge":  # latencies past fp16's 65504: the saturated keys
        g = synth.geometric_complete_ish(V=1500, A=200)
        g.latency = g.latency * 1000.0
    elif case == "ties":
        g = synth.integer_grid(rows=11, cols=12, seed=6)
    else:
        rng = np.random.default_rng(5)
        g = synth.random_sparse(V=170, avg_deg=8, seed=7, vloss=rng.uniform(0, 0.1, 170))
        g.prefer_direct = True
    st = compare(g, layout="dense", dense_w16=1)
    assert st["dense"] == 1 and st["full_sweeps"] > 0


@pytest.mark.parametrize("layout", ["csr", "dense"])
def test_host_rows_interleaved_lat_rel(layout):
    """SHADOWTOPO_MEM_HOST_LR (the shim's per-packet layout): {lat, rel} pairs interleaved in
    one host array, page-locked (pipelined copy over several groups) and pageable, identical
    to the separate arrays; a replayed (tie) source's rows too"""
    g = synth.integer_grid(rows=12, cols=12, seed=3) if layout == "csr" else synth.geometric_complete_ish(V=600, A=150)
    eng = E.Engine.from_synth(g, layout=layout)
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_BATCHES_IN_FLIGHT, 1)
    lat, rel, _, kind = eng.compute_rows()
    for pinned in (True, False):
        lr, kl = eng.compute_rows_lr(pinned=pinned)
        assert np.array_equal(lr[:, :, 0].view(np.uint64), lat.view(np.uint64))
        assert np.array_equal(lr[:, :, 1].view(np.uint64), rel.view(np.uint64))
        assert np.array_equal(kl, kind)
        a, b = 5, len(g.attached) - 3
        lr2, _ = eng.compute_rows_lr(a, b, pinned=pinned)
        assert np.array_equal(lr2[:, :, 0].view(np.uint64), lat[a:b].view(np.uint64))
    if layout == "csr":
        assert eng.stats()["replayed_sources"] > 0
    eng.close()


@pytest.mark.parametrize("spec", [0, 1, 2, 4])
@pytest.mark.parametrize("case", ["geometric", "ties", "directed", "over_thresh"])
def test_dense_rounds_without_read_back(case, spec):
    """OPT_DENSE_SPEC: the first rounds enqueued back to back with no host read-back of their
    change counts (a round decided blind runs the delta kernel over every batch that changed,
    or a full sweep when delta rounds are off) give the oracle's matrices, bit for bit, and
    fewer host synchronisations; over_thresh: a 1-per-mille delta threshold, so the batches
    that the host would full-sweep again after round 0 take a blind delta round instead"""
    permille = 125
    if case == "geometric":
        g = synth.geometric_complete_ish(V=900, A=200)
    elif case == "ties":
        g = synth.integer_grid(rows=11, cols=12, seed=6)
    elif case == "directed":
        g = synth.random_sparse(V=260, avg_deg=5, seed=9, directed=True)
    else:
        g = synth.geometric_complete_ish(V=700, A=150, drop=0.3)
        permille = 1
    st = compare(g, layout="dense", dense_spec=spec, delta_permille=permille)
    assert st["dense"] == 1
    if spec:
        assert st["host_syncs"] < st["rounds"] + st["groups"], st
    st0 = compare(g, layout="dense", dense_spec=spec, delta_permille=0)  # full sweeps only
    assert st0["delta_sweeps"] == 0


@pytest.mark.parametrize("on", [0, 1])
@pytest.mark.parametrize("spec", [0, 2])
@pytest.mark.parametrize("case", ["geometric", "ties", "vloss_multigraph", "several_groups"])
def test_dense_speculative_compose(case, spec, on):
    """OPT_SPEC_COMPOSE: the compose enqueued behind every dense delta round before its
    read-back, kept when that round changed nothing and redone (masks and error word reset)
    when it did -- including path walks over a state that had not converged yet (vertex loss,
    a multigraph), whose error word must not survive -- bit-exact against the oracle"""
    if case == "geometric":
        g = synth.geometric_complete_ish(V=900, A=200)
    elif case == "ties":
        g = synth.integer_grid(rows=11, cols=12, seed=6)
    elif case == "several_groups":
        g = synth.geometric_complete_ish(V=700, A=300, drop=0.2)
    else:
        g = synth.random_sparse(V=220, avg_deg=8, seed=17, vloss=np.where(np.arange(220) % 3 == 0, 0.03, np.nan))
        rng = np.random.default_rng(4)
        pick = rng.choice(np.nonzero(g.src != g.dst)[0], 30, replace=False)
        g.src = np.concatenate([g.src, g.dst[pick]])
        g.dst = np.concatenate([g.dst, g.src[pick]])
        g.latency = np.concatenate([g.latency, g.latency[pick] * rng.uniform(0.5, 1.5, 30)])
        g.packetloss = np.concatenate([g.packetloss, rng.uniform(0, 0.05, 30)])
    opts = dict(batches_in_flight=2) if case == "several_groups" else {}
    st = compare(g, layout="dense", dense_spec=spec, spec_compose=on, **opts)
    assert st["dense"] == 1
    if not on:
        assert st["spec_composes"] == 0 and st["spec_composes_lost"] == 0
    elif case != "ties":
        assert st["spec_composes"] > 0, st


@pytest.mark.parametrize("tb", [1, 2, 4])
@pytest.mark.parametrize("case", ["geometric", "geometric_odd", "ties"])
def test_dense_batches_per_wave(case, tb):
    """OPT_DENSE_BATCHES_PER_WAVE: the chunk loop filtering 1, 2 or 4 batches per wave against
    one staged W32 slab (the exact pass then one batch per wave, from the per-batch hit log),
    with an odd batch count, bit for bit the oracle's matrices"""
    if case == "geometric":
        g = synth.geometric_complete_ish(V=900, A=256)
    elif case == "geometric_odd":
        g = synth.geometric_complete_ish(V=611, A=150)  # 3 batches: a half-empty wave group
    else:
        g = synth.integer_grid(rows=11, cols=12, seed=6)
    st = compare(g, layout="dense", dense_batches_per_wave=tb)
    assert st["dense"] == 1 and st["full_sweeps"] >= 1


@pytest.mark.parametrize("case", ["geometric", "vloss_prefer", "ties_dense", "odd_block"])
def test_row_codec_round_trip(case):
    """the row exchange codec (shadowtopo_pack_rows / unpack_rows): device rows packed by one
    engine and unpacked by ANOTHER engine built from the same graph (another rank's replica)
    come back bit for bit, equal to the oracle's; the single-arc pairs of a geometric graph
    are rebuilt, not sent (payload < 1/4 of the raw rows)"""
    import torch
    rng = np.random.default_rng(9)
    if case == "geometric":
        g = synth.geometric_complete_ish(V=700, A=200)
    elif case == "vloss_prefer":
        g = synth.geometric_complete_ish(V=400, A=150)
        g.vertex_packetloss = np.where(rng.random(400) < 0.3, 0.01, np.nan)
        g.prefer_direct = True
    elif case == "ties_dense":
        g = synth.integer_grid(rows=11, cols=12, seed=6)
    else:
        g = synth.geometric_complete_ish(V=333, A=77, drop=0.3)
    lat_o, rel_o, hops_o, _, _ = oracle_matrix(g)
    dev = torch.device("cuda:0")
    engs = [E.Engine.from_synth(g, layout="dense") for _ in range(2)]
    for e in engs:
        e.set_attached(g.attached)
    A = len(g.attached)
    a, z = (3, A - 5) if case == "odd_block" else (0, A)
    n = z - a
    lat = torch.empty((n, A), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    hops = torch.empty((n, A), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    engs[0].compute_rows_device(a, z, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=s)
    cap = E.Engine.packed_capacity(n, A)
    buf = torch.empty(cap, dtype=torch.uint8, device=dev)
    nbytes = engs[0].pack_rows(a, z, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), buf.data_ptr(), cap, stream=s)
    assert 0 < nbytes <= cap
    out = [torch.full_like(lat, -7.0), torch.full_like(rel, -7.0), torch.full_like(hops, -7)]
    engs[1].unpack_rows(a, z, buf.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), stream=s)
    torch.cuda.synchronize(dev)
    assert_bitexact("latency", out[0].cpu().numpy(), lat_o[a:z])
    assert_bitexact("reliability", out[1].cpu().numpy(), rel_o[a:z])
    assert_bitexact("hops", out[2].cpu().numpy().astype(np.uint32), hops_o[a:z])
    st = engs[0].stats()
    assert st["packed_pairs"] == n * A
    if case == "geometric":
        assert nbytes * 4 < n * A * 20, (nbytes, n * A * 20)
    for e in engs:
        e.close()


def test_row_codec_needs_a_dense_engine():
    g = synth.random_sparse(V=200, avg_deg=4, seed=3, A=50)
    eng = E.Engine.from_synth(g, layout="csr")
    eng.set_attached(g.attached)
    with pytest.raises(E.ShadowTopoError):
        eng.pack_rows(0, 1, 0, 0, 0, 0, E.Engine.packed_capacity(1, 50))
    eng.close()


@pytest.mark.parametrize("parts", [1, 2, 3, 4])
@pytest.mark.parametrize("case", ["geometric", "geometric_odd", "ties", "vloss_prefer"])
def test_dense_sweep_parts(case, parts):
    """OPT_SWEEP_PARTS: the pruned sweep's batches in 1 / 2 / 4 parts, each on its own stream
    (chunk loop and exact pass per part, the parts overlapping): the oracle's matrices bit for
    bit, with fewer batches than parts too"""
    rng = np.random.default_rng(3)
    if case == "geometric":
        g = synth.geometric_complete_ish(V=900, A=330)       # 6 batches
    elif case == "geometric_odd":
        g = synth.geometric_complete_ish(V=611, A=100)       # 2 batches: 4 parts clamp to 2
    elif case == "ties":
        g = synth.integer_grid(rows=14, cols=15, seed=6)
    else:
        g = synth.geometric_complete_ish(V=500, A=200)
        g.vertex_packetloss = np.where(rng.random(500) < 0.3, 0.01, np.nan)
        g.prefer_direct = True
    compare(g, layout="dense", sweep_parts=parts)


@pytest.mark.parametrize("chain", [0, 1])
@pytest.mark.parametrize("parts,spec", [(2, 1), (2, 2), (3, 2), (4, 2), (2, 4), (4, 4)])
@pytest.mark.parametrize("case", ["geometric", "geometric7", "ties", "vloss_prefer"])
def test_chained_part_rounds(case, parts, spec, chain):
    """OPT_CHAIN_PARTS: the read-back-free delta rounds (OPT_DENSE_SPEC of them) enqueued on
    each sweep part's stream behind its share of the sweep, one join before the read-back:
    pruned, sparse and plain delta kinds on per-part pools, cnt rows, bounds and chunk masks
    all meet the oracle bit for bit (and the unchained order with them)"""
    rng = np.random.default_rng(11)
    if case == "geometric":
        g = synth.geometric_complete_ish(V=900, A=330)       # 6 batches
    elif case == "geometric7":
        g = synth.geometric_complete_ish(V=900, A=430)       # 7 batches: two parts of 4 + 3 (OPT part-0 share)
    elif case == "ties":
        g = synth.integer_grid(rows=14, cols=15, seed=8)
    else:
        g = synth.geometric_complete_ish(V=500, A=200)
        g.vertex_packetloss = np.where(rng.random(500) < 0.3, 0.01, np.nan)
        g.prefer_direct = True
    compare(g, layout="dense", sweep_parts=parts, dense_spec=spec, chain_parts=chain)


@pytest.mark.parametrize("live", [0, 1])
def test_chained_part_rounds_delta_kinds(live):
    """chained rounds with the live-chunk lists forced on (every blind round sparse) or off
    (the pruned round, then plain ones): both kinds' per-part offsets"""
    g = synth.geometric_complete_ish(V=700, A=260)
    compare(g, layout="dense", sweep_parts=2, dense_spec=3, chain_parts=1, delta_live=live)


def _vloss_graph(V=300, seed=31):
    rng = np.random.default_rng(seed)
    vl = np.where(rng.random(V) < 0.5, rng.uniform(0, 0.1, V), np.nan)
    return synth.random_sparse(V=V, avg_deg=4, seed=seed, vloss=vl)


@pytest.mark.parametrize("layout", ["csr", "dense"])
@pytest.mark.parametrize("mode", [1, 2])
def test_scrambled_tree_reports_an_error(mode, layout):
    """compose's path walks (targets with vertex loss) on predecessor records that are no
    longer a tree -- arcs past the range (1), or every vertex's first in-arc (2) -- end in
    SHADOWTOPO_EINTERNAL, not a device fault; the engine then computes correctly"""
    g = _vloss_graph()
    eng = E.Engine.from_synth(g, layout=layout)
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_TEST_SCRAMBLE_TREE, mode)
    with pytest.raises(E.ShadowTopoError, match="error -5: a path walk left the predecessor tree"):
        eng.compute_rows()
    eng.set_option(E.OPT_TEST_SCRAMBLE_TREE, 0)
    lat, rel, hops, kind = eng.compute_rows()
    eng.close()
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                       ("reliability", rel, orel)):
        assert_bitexact(name, x, y)


@pytest.mark.parametrize("worklist", [1, 2])
@pytest.mark.parametrize("mode", [1, 2])
def test_scrambled_lean_state_reports_an_error(mode, worklist):
    """the lean rounds' predecessor state (P32) scrambled before the walks, over several batches
    (batch >= 1 is where r05r's fault was: a tree-record pointer formed from the absent pool):
    k_walk_lean's range checks end the call in SHADOWTOPO_EINTERNAL, not a device fault, and
    the same engine then computes the oracle's matrices"""
    g = _vloss_graph(V=600, seed=41)
    g.attached = np.arange(0, g.n, 3, dtype=np.int32)  # 200 sources: 4 batches
    eng = E.Engine.from_synth(g, layout="csr")
    eng.set_option(E.OPT_CSR_LEAN, 1)
    eng.set_option(E.OPT_WORKLIST, worklist)
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_TEST_SCRAMBLE_TREE, mode)
    with pytest.raises(E.ShadowTopoError, match="error -5"):
        eng.compute_rows()
    eng.set_option(E.OPT_TEST_SCRAMBLE_TREE, 0)
    lat, rel, hops, kind = eng.compute_rows()
    st = eng.stats()
    eng.close()
    assert st["lean_groups"] >= 1
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                       ("reliability", rel, orel)):
        assert_bitexact(name, x, y)


@pytest.mark.parametrize("layout", ["csr", "dense"])
def test_unconverged_state_composes_without_fault(layout):
    """the iteration guard tripped after one round (OPT_MAX_ROUNDS 1) with the testing option
    that composes the state it stopped at: the bounded walks read a non-converged state and
    the call fails with SHADOWTOPO_EINTERNAL; the same engine then computes correctly"""
    g = _vloss_graph(V=400, seed=33)
    eng = E.Engine.from_synth(g, layout=layout)
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_MAX_ROUNDS, 1)
    eng.set_option(E.OPT_TEST_UNCONVERGED, 1)
    with pytest.raises(E.ShadowTopoError, match="error -5"):
        eng.compute_rows()
    eng.set_option(E.OPT_MAX_ROUNDS, 0)
    eng.set_option(E.OPT_TEST_UNCONVERGED, 0)
    lat, rel, hops, kind = eng.compute_rows()
    eng.close()
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                       ("reliability", rel, orel)):
        assert_bitexact(name, x, y)


@pytest.mark.parametrize("shape", [1, 2])
def test_long_paths_walk_in_segments(shape):
    """vertex-loss targets whose paths have more hops than one walk segment (16 arcs): a
    path graph (every vertex on one chain, hops up to V - 1) with vertex loss everywhere"""
    V = 90
    src = np.arange(V - 1, dtype=np.int32)
    dst = np.arange(1, V, dtype=np.int32)
    rng = np.random.default_rng(4)
    g = synth._finish("chain", V, src, dst, rng.uniform(1, 5, V - 1), rng.uniform(0, 0.05, V - 1),
                      np.arange(0, V, 3, dtype=np.int32))
    g.vertex_packetloss = rng.uniform(0, 0.05, V)
    compare(g, walk_tpw=shape)
    _, _, hops, _, _ = engine_matrix(g)
    assert hops.max() > 48


def test_pool_enomem_retry():
    """a batch-pool allocation that fails after the budget was computed (another engine or
    process took the HBM: OPT_TEST_POOL_ENOMEM injects it) is retried with pools sized from
    a fresh free-memory query, and the results are the oracle's"""
    g = synth.random_sparse(V=400, avg_deg=4, seed=35)
    eng = E.Engine.from_synth(g)
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_TEST_POOL_ENOMEM, 1)
    lat, rel, hops, kind = eng.compute_rows()
    st = eng.stats()
    eng.close()
    assert st["pool_allocs"] == 2, st["pool_allocs"]
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                       ("reliability", rel, orel)):
        assert_bitexact(name, x, y)


@pytest.mark.parametrize("layout", ["csr", "dense"])
def test_alternating_attached_sets(layout):
    """set_attached with a new list before every computation (bench --fresh-attach): the self
    rule, source order and relaxation view of each set are rebuilt, and every matrix is the
    oracle's; the self rule runs inside each computation"""
    g = synth.random_sparse(V=500, avg_deg=5, seed=37, A=120) if layout == "csr" else \
        synth.geometric_complete_ish(V=700, A=120)
    rng = np.random.default_rng(5)
    other = np.sort(rng.choice(g.n, size=len(g.attached), replace=False)).astype(np.int32)
    eng = E.Engine.from_synth(g, layout=layout)
    for k, att in enumerate([g.attached, other, g.attached, other]):
        eng.set_attached(att)
        lat, rel, hops, kind = eng.compute_rows()
        g.attached = att
        olat, orel, ohops, okind, og = oracle_matrix(g)
        og.close()
        for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                           ("reliability", rel, orel)):
            assert_bitexact(f"set {k} {name}", x, y)
    st = eng.stats()
    eng.close()
    assert st["self_paths"] == 4 * len(other)


@pytest.mark.parametrize("parts", [2, 3, 4])
@pytest.mark.parametrize("case", ["geometric", "ties"])
def test_heavy_first_sweep_order(case, parts):
    """OPT_HEAVY_FIRST: each part's chunk-loop blocks in the order of the chunk counts the
    previous sweep of the same shape recorded (k_heavy_order, ping-pong order buffers): the
    first computation runs in grid order, the next ones heavy-first, every one the oracle's
    matrices bit for bit, and the same as with the order off; a new attached set (another
    shape) falls back to grid order"""
    g = synth.geometric_complete_ish(V=900, A=330) if case == "geometric" else synth.integer_grid(rows=14, cols=15, seed=6)
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    eng = E.Engine.from_synth(g, layout="dense")
    eng.set_option(E.OPT_SWEEP_PARTS, parts)
    eng.set_attached(g.attached)
    for step in range(4):
        eng.set_option(E.OPT_HEAVY_FIRST, 0 if step == 2 else 1)
        lat, rel, hops, kind = eng.compute_rows()
        for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                           ("reliability", rel, orel)):
            assert_bitexact(f"step {step} {name}", x, y)
    sub = g.attached[: len(g.attached) // 2]
    eng.set_attached(sub)
    lat, rel, hops, kind = eng.compute_rows()
    eng.close()
    assert_bitexact("new set latency", lat, olat[: len(sub), : len(sub)])
    assert_bitexact("new set hops", hops, ohops[: len(sub), : len(sub)])


def test_late_walk_table_keeps_heavy_first_buffers():
    """a dense engine runs parted heavy-first sweeps on a loss-free attached set (the chunk-count
    and order buffers are allocated), then set_attached adds targets with vertex loss, so the
    walk's per-arc table is allocated for the first time: the heavy-first buffers must survive
    that allocation (r05 advisor: a pasted loop freed them there), every matrix is the oracle's
    and close() frees each buffer once"""
    g = synth.geometric_complete_ish(V=900, A=330)
    rng = np.random.default_rng(12)
    vl = np.full(g.n, np.nan)
    lossy = np.setdiff1d(np.arange(g.n), g.attached)[:40]
    vl[lossy] = rng.uniform(0.0, 0.05, len(lossy))
    g.vertex_packetloss = vl
    eng = E.Engine.from_synth(g, layout="dense")
    eng.set_option(E.OPT_SWEEP_PARTS, 2)
    eng.set_option(E.OPT_HEAVY_FIRST, 1)
    sets = [g.attached, np.sort(np.concatenate([g.attached[:300], lossy[:30]])).astype(np.int32)]
    for k, att in enumerate([sets[0], sets[0], sets[1], sets[1], sets[0]]):
        eng.set_attached(att)
        lat, rel, hops, kind = eng.compute_rows()
        g.attached = att
        olat, orel, ohops, okind, og = oracle_matrix(g)
        og.close()
        for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                           ("reliability", rel, orel)):
            assert_bitexact(f"set {k} {name}", x, y)
    st = eng.stats()
    eng.close()
    assert st["walk_targets"] == 0  # the last set is loss-free again


@pytest.mark.parametrize("case", ["geometric", "ties", "vloss_prefer"])
def test_dense_sweep_glds_staging(case):
    """OPT_SWEEP_GLDS: the pruned chunk loop staged by LDS-DMA (global_load_lds) or through
    registers (the default), two sweep parts, heavy-first from the second computation: the
    oracle's matrices bit for bit every time"""
    if case == "ties":
        g = synth.integer_grid(rows=14, cols=15, seed=6)
    elif case == "vloss_prefer":
        g = synth.geometric_complete_ish(V=600, A=200)
        rng = np.random.default_rng(3)
        g.vertex_packetloss = np.where(rng.random(g.n) < 0.3, rng.uniform(0, 0.05, g.n), np.nan)
        g.prefer_direct = True
    else:
        g = synth.geometric_complete_ish(V=900, A=330)
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    eng = E.Engine.from_synth(g, layout="dense")
    eng.set_attached(g.attached)
    for step in range(4):
        eng.set_option(E.OPT_SWEEP_GLDS, 0 if step == 2 else 1)  # register staging (the default) once, between
        lat, rel, hops, kind = eng.compute_rows()
        for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                           ("reliability", rel, orel)):
            assert_bitexact(f"step {step} {name}", x, y)
    eng.close()


@pytest.mark.parametrize("case", ["geometric", "ties", "vloss_prefer", "directed"])
def test_dense_sweep_refilter(case):
    """OPT_SWEEP_REFILTER: the exact pass drops the logged rows that no lane passes under the
    chunk loop's final f32 thresholds; every computation (grid order, then heavy-first, with
    and without the refilter) equals the oracle's matrices bit for bit"""
    if case == "ties":
        g = synth.integer_grid(rows=14, cols=15, seed=6)
    elif case == "directed":
        g = synth.random_sparse(V=300, avg_deg=40, seed=9, directed=True)
    elif case == "vloss_prefer":
        g = synth.geometric_complete_ish(V=600, A=200)
        rng = np.random.default_rng(3)
        g.vertex_packetloss = np.where(rng.random(g.n) < 0.3, rng.uniform(0, 0.05, g.n), np.nan)
        g.prefer_direct = True
    else:
        g = synth.geometric_complete_ish(V=900, A=330)
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    eng = E.Engine.from_synth(g, layout="dense")
    eng.set_attached(g.attached)
    for step in range(4):
        eng.set_option(E.OPT_SWEEP_REFILTER, 0 if step == 2 else 1)
        lat, rel, hops, kind = eng.compute_rows()
        for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                           ("reliability", rel, orel)):
            assert_bitexact(f"step {step} {name}", x, y)
    eng.close()


@pytest.mark.parametrize("mode", ["chained", "host_rounds", "full_sweeps"])
@pytest.mark.parametrize("case", ["geometric", "ties", "vloss_prefer", "directed"])
def test_dense_seed_skip(case, mode):
    """OPT_SEED_SKIP: round 0's exact pass leaves the pairs whose seed candidate won untainted
    unread (their stored state is k_seed_dense_t's); later full sweeps (OPT_DELTA_PERMILLE 0:
    every round a full sweep) must not.  Chained part rounds, host-driven rounds and full
    sweeps only, each with and without the skip and across two attached sets, equal the
    oracle's matrices bit for bit"""
    if case == "ties":
        g = synth.integer_grid(rows=14, cols=15, seed=6)
    elif case == "directed":
        g = synth.random_sparse(V=300, avg_deg=40, seed=9, directed=True)
    elif case == "vloss_prefer":
        g = synth.geometric_complete_ish(V=600, A=200)
        rng = np.random.default_rng(3)
        g.vertex_packetloss = np.where(rng.random(g.n) < 0.3, rng.uniform(0, 0.05, g.n), np.nan)
        g.prefer_direct = True
    else:
        g = synth.geometric_complete_ish(V=900, A=330)
    other = np.sort(np.random.default_rng(21).choice(g.n, size=len(g.attached), replace=False)).astype(np.int32)
    eng = E.Engine.from_synth(g, layout="dense")
    if mode == "host_rounds":
        eng.set_option(E.OPT_DENSE_SPEC, 0)
    elif mode == "full_sweeps":
        eng.set_option(E.OPT_DELTA_PERMILLE, 0)
    for att in (g.attached, other):
        g.attached = att
        olat, orel, ohops, okind, og = oracle_matrix(g)
        og.close()
        eng.set_attached(att)
        for skip in (1, 0, 1):
            eng.set_option(E.OPT_SEED_SKIP, skip)
            lat, rel, hops, kind = eng.compute_rows()
            for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                               ("reliability", rel, orel)):
                assert_bitexact(f"skip {skip} {name}", x, y)
    eng.close()


@pytest.mark.parametrize("case", ["geometric", "ties", "vloss_prefer", "directed", "wide_latency"])
def test_dense_delta_w16(case):
    """OPT_DELTA_W16: the pruned delta rounds filter against fp16 slabs (W rounded toward
    -inf); with and without it, chained and after the join, the matrices equal the oracle's
    bit for bit (wide_latency: weights over several decades, where fp16 is coarsest)"""
    if case == "ties":
        g = synth.integer_grid(rows=14, cols=15, seed=6)
    elif case == "directed":
        g = synth.random_sparse(V=300, avg_deg=40, seed=9, directed=True)
    elif case == "vloss_prefer":
        g = synth.geometric_complete_ish(V=600, A=200)
        rng = np.random.default_rng(3)
        g.vertex_packetloss = np.where(rng.random(g.n) < 0.3, rng.uniform(0, 0.05, g.n), np.nan)
        g.prefer_direct = True
    elif case == "wide_latency":
        g = synth.geometric_complete_ish(V=700, A=250)
        g.latency = g.latency * np.exp(np.random.default_rng(8).uniform(0.0, 9.0, len(g.latency)))
    else:
        g = synth.geometric_complete_ish(V=900, A=330)
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    eng = E.Engine.from_synth(g, layout="dense")
    eng.set_attached(g.attached)
    for w16, chain in ((1, 1), (0, 1), (1, 0)):
        eng.set_option(E.OPT_DELTA_W16, w16)
        eng.set_option(E.OPT_CHAIN_PARTS, chain)
        lat, rel, hops, kind = eng.compute_rows()
        for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                           ("reliability", rel, orel)):
            assert_bitexact(f"w16 {w16} chain {chain} {name}", x, y)
    eng.close()


@pytest.mark.parametrize("glds", [0, 1])
@pytest.mark.parametrize("case", ["geometric", "ties", "vloss_prefer"])
def test_dense_sweep_eight_wave_blocks(case, glds):
    """OPT_SWEEP_WAVES 8: the chunk loop in 8-wave blocks (64 destinations per staged chunk),
    the exact pass in 4-wave blocks reading the same per-wave hit logs; grid order, then
    heavy-first (another block shape: its own order), then 4-wave blocks again -- the oracle's
    matrices bit for bit every time"""
    if case == "ties":
        g = synth.integer_grid(rows=14, cols=15, seed=6)
    elif case == "vloss_prefer":
        g = synth.geometric_complete_ish(V=600, A=200)
        rng = np.random.default_rng(3)
        g.vertex_packetloss = np.where(rng.random(g.n) < 0.3, rng.uniform(0, 0.05, g.n), np.nan)
        g.prefer_direct = True
    else:
        g = synth.geometric_complete_ish(V=900, A=330)
    olat, orel, ohops, okind, og = oracle_matrix(g)
    og.close()
    eng = E.Engine.from_synth(g, layout="dense")
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_SWEEP_GLDS, glds)
    for step in range(4):
        eng.set_option(E.OPT_SWEEP_WAVES, 4 if step == 3 else 8)
        lat, rel, hops, kind = eng.compute_rows()
        for name, x, y in (("kind", kind, okind), ("latency", lat, olat), ("hops", hops, ohops),
                           ("reliability", rel, orel)):
            assert_bitexact(f"step {step} {name}", x, y)
    eng.close()
