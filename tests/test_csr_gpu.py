"""CSR relaxation rounds (k_relax over the whole grid, k_relax_wl / k_relax_wlp over frontier
worklists, host- or device-driven, 1-D or 2-D grids, one or several batch groups) against
the oracle and against each other.  Same bar as test_engine_gpu.py: bit-exact latency, hops,
kind and reliability; every schedule must reach the same fixed point."""
import numpy as np
import pytest

from paritylib import compare
from shadow_amd import engine as E
from shadow_amd import synth

pytestmark = pytest.mark.gpu


def _case(case):
    if case == "sparse":
        return synth.random_sparse(V=400, avg_deg=5, seed=31)
    if case == "directed":
        return synth.random_sparse(V=300, avg_deg=4, seed=32, directed=True)
    if case == "ties":
        return synth.integer_grid(rows=12, cols=12, seed=5)
    if case == "int_random":
        return synth.random_sparse(V=300, avg_deg=5, seed=33, int_lat=True)
    if case == "vloss_prefer":
        rng = np.random.default_rng(7)
        g = synth.random_sparse(V=250, avg_deg=6, seed=34, vloss=np.where(rng.random(250) < 0.5, 0.02, np.nan))
        g.prefer_direct = True
        return g
    if case == "no_loops":
        return synth.random_sparse(V=250, avg_deg=3, seed=36, loops=False)
    g = synth.random_sparse(V=150, avg_deg=4, seed=35)  # multigraph: parallel edges
    rng = np.random.default_rng(3)
    pick = rng.choice(np.nonzero(g.src != g.dst)[0], 40, replace=False)
    g.src = np.concatenate([g.src, g.dst[pick]])
    g.dst = np.concatenate([g.dst, g.src[pick]])
    g.latency = np.concatenate([g.latency, g.latency[pick] * rng.uniform(0.3, 1.7, 40)])
    g.packetloss = np.concatenate([g.packetloss, rng.uniform(0, 0.05, 40)])
    return g


CASES = ["sparse", "directed", "ties", "int_random", "vloss_prefer", "no_loops", "multigraph"]


# the sparse round state: the tree fold inside the rounds, lean rounds + a walk per pair, and
# lean rounds whose visits re-read only the tails changed since (OPT_CSR_INCREMENTAL; 1: every
# vertex with more than one in-arc, so the small graphs here take the incremental visit)
MODES = {"tree": dict(csr_lean=0), "lean": dict(csr_lean=1, csr_incremental=0),
         "inc": dict(csr_lean=1, csr_incremental=1)}


@pytest.mark.parametrize("lean", list(MODES))
@pytest.mark.parametrize("worklist", [1, 2])
@pytest.mark.parametrize("case", CASES)
def test_csr_rounds(case, worklist, lean):
    """default schedule (worklists when under half the pairs are active) and always-worklist,
    in every round-state mode"""
    g = _case(case)
    st = compare(g, layout="csr", worklist=worklist, **MODES[lean])
    assert st["dense"] == 0
    assert (st["lean_groups"] > 0) == (lean != "tree")


def test_option_ranges():
    """the r05 options take their documented values and reject the rest (SHADOWTOPO_EINVAL)"""
    g = _case("sparse")
    eng = E.Engine.from_synth(g, layout="csr")
    good = {E.OPT_CSR_INCREMENTAL: (0, 1, 32, 1 << 20), E.OPT_SPEC_COMPOSE: (0, 1), E.OPT_SPIN_US: (0, 200, 20000),
            E.OPT_HOST_GROUPS: (0, 1, 4), E.OPT_CSR_LEAN: (0, 1, 2), E.OPT_HEAVY_FIRST: (0, 1),
            E.OPT_WALK_TPW: (1, 2, 4), E.OPT_PART0_PERMILLE: (1, 562, 999)}
    bad = {E.OPT_CSR_INCREMENTAL: (-1, (1 << 20) + 1), E.OPT_SPEC_COMPOSE: (2, -1), E.OPT_SPIN_US: (-1, 10_000_001),
           E.OPT_HOST_GROUPS: (-1, 1025), E.OPT_CSR_LEAN: (3,), E.OPT_HEAVY_FIRST: (2,), E.OPT_WALK_TPW: (0, 5),
           E.OPT_PART0_PERMILLE: (0, 1000)}
    for k, vals in good.items():
        for v in vals:
            eng.set_option(k, v)
    for k, vals in bad.items():
        for v in vals:
            with pytest.raises(E.ShadowTopoError):
                eng.set_option(k, v)
    eng.close()


def test_csr_removed_variants_rejected():
    g = _case("sparse")
    eng = E.Engine.from_synth(g, layout="csr")
    eng.set_option(E.OPT_CSR_VARIANT, E.CSR_FULL)
    eng.set_option(E.OPT_CSR_VARIANT, E.CSR_PUSH)  # the push rounds (undirected graphs)
    for v in (0, 3, 4):
        with pytest.raises(E.ShadowTopoError):
            eng.set_option(E.OPT_CSR_VARIANT, v)
    eng.close()


@pytest.mark.parametrize("case", CASES)
def test_csr_full_grid_without_worklists(case):
    """the default FULL rounds run over compacted frontier worklists; the one-wave-per-pair
    grid must give the same matrices"""
    g = _case(case)
    compare(g, layout="csr", worklist=0)
    compare(g, layout="csr", worklist=1, batches_in_flight=2)


@pytest.mark.parametrize("lean", list(MODES))
@pytest.mark.parametrize("worklist", [0, 1, 2])
def test_csr_two_dimensional_grids(worklist, lean):
    """grids past 2^24 blocks (C5: 102 batches x 868k vertices = 22M blocks of 256) go 2-D
    (grid_of / flat_block: a 1-D launch's 32-bit work-item count would wrap and drop
    blocks, and a round that dropped a batch could end the iteration early); forcing the
    2-D form on every launch of a small graph must give the same matrices"""
    g = synth.random_sparse(V=400, avg_deg=5, seed=38)
    compare(g, layout="csr", worklist=worklist, grid_x=64, **MODES[lean])


@pytest.mark.parametrize("lean", list(MODES))
@pytest.mark.parametrize("worklist", [0, 1])
def test_csr_several_groups(worklist, lean):
    g = synth.random_sparse(V=500, avg_deg=4, seed=37)
    compare(g, layout="csr", batches_in_flight=3, worklist=worklist, **MODES[lean])  # 8 batches -> 3 groups


@pytest.mark.parametrize("case", ["sparse", "ties", "vloss_prefer", "multigraph", "directed"])
def test_lean_rounds_long_paths_and_auto(case):
    """lean rounds (OPT_CSR_LEAN 1) on a path-heavy graph (a chain with chords: hop counts far
    past one walk segment) and the automatic choice on a graph with many arcs per attached
    vertex (few attached targets: lean), both against the oracle"""
    g = _case(case)
    rng = np.random.default_rng(11)
    g.attached = np.sort(rng.choice(g.n, size=max(2, g.n // 40), replace=False)).astype(np.int32)
    st = compare(g, layout="csr")  # auto: arcs >= 32 x attached
    assert st["lean_groups"] > 0
    V = 200
    src = np.concatenate([np.arange(V - 1), rng.integers(0, V, 6)]).astype(np.int32)
    dst = np.concatenate([np.arange(1, V), rng.integers(0, V, 6)]).astype(np.int32)
    keep = src != dst
    chain = synth._finish("chain", V, src[keep], dst[keep], rng.uniform(1, 5, keep.sum()),
                          rng.uniform(0, 0.05, keep.sum()), np.arange(0, V, 7, dtype=np.int32))
    chain.vertex_packetloss = np.where(rng.random(V) < 0.5, rng.uniform(0, 0.05, V), np.nan)
    compare(chain, layout="csr", csr_lean=1)
    compare(chain, layout="csr", csr_lean=1, csr_incremental=1)


def _long_chain(V, seed, chords=2):
    """a path with a few chords: the rounds run about as many rounds as the path is long"""
    rng = np.random.default_rng(seed)
    src = np.concatenate([np.arange(V - 1), rng.integers(0, V, chords)]).astype(np.int32)
    dst = np.concatenate([np.arange(1, V), rng.integers(0, V, chords)]).astype(np.int32)
    keep = src != dst
    lat = rng.uniform(1, 5, keep.sum())
    lat[: V // 3] = np.round(lat[: V // 3])  # integer latencies on a stretch: ties through the chords
    return synth._finish("chain", V, src[keep], dst[keep], lat, rng.uniform(0, 0.05, keep.sum()),
                         np.arange(0, V, 7, dtype=np.int32))


@pytest.mark.parametrize("sched", ["grid", "worklist", "device"])
def test_incremental_rounds_past_stamp_wrap(sched):
    """incremental lean rounds (OPT_CSR_INCREMENTAL) stamp each change with the round mod 256:
    on a 1200-vertex chain the rounds run past the wrap (a stale stamp that matches again
    only costs a re-read), over every schedule and several batch groups, bit-exact against
    the oracle and the non-incremental lean rounds"""
    g = _long_chain(1200, seed=12)
    opts = {"grid": dict(worklist=0), "worklist": dict(worklist=1, device_rounds=0),
            "device": dict(worklist=1, device_rounds=2)}[sched]
    st = compare(g, layout="csr", csr_lean=1, csr_incremental=1, batches_in_flight=1, **opts)
    assert st["rounds"] > 300 and st["lean_groups"] > 1, (st["rounds"], st["lean_groups"])
    compare(g, layout="csr", csr_lean=1, csr_incremental=0, batches_in_flight=1, **opts)


@pytest.mark.parametrize("case", ["ties", "sparse", "int_random", "directed"])
def test_csr_schedules_same_fixed_point(case):
    """Full rows (sssp) from the grid, worklist and device-driven schedules: distances
    bit-exact, tie flags identical, predecessor and hops identical wherever no heap-order
    tie is involved."""
    g = _case(case)
    srcs = np.arange(0, g.n, 2, dtype=np.int32)
    outs = []
    for wl, devr in ((0, 0), (1, 0), (2, 0), (1, 2)):
        eng = E.Engine.from_synth(g, layout="csr")
        eng.set_option(E.OPT_WORKLIST, wl)
        eng.set_option(E.OPT_DEVICE_ROUNDS, devr)
        outs.append(eng.sssp(srcs))
        eng.close()
    d0, p0, h0, t0 = outs[0]
    for d1, p1, h1, t1 in outs[1:]:
        assert np.array_equal(d0.view(np.uint64), d1.view(np.uint64))
        assert np.array_equal(t0, t1)
        ok = t0 == 0
        assert np.array_equal(p0[ok], p1[ok]) and np.array_equal(h0[ok], h1[ok])
    if case in ("ties", "int_random"):
        assert (t0 != 0).any()


@pytest.mark.parametrize("case", ["knn", "ties", "directed"])
def test_source_order_same_matrix(case):
    """OPT_SOURCE_ORDER only changes which sources share a wave: the matrix is bit-identical
    to attach-order batching (and to the oracle), for a geographic graph the locality order
    visits fewer (vertex, batch) pairs, and a row range that is not the whole attached set
    is permuted within itself."""
    if case == "knn":
        g = synth.knn_geographic(V=1500, k=8)
    elif case == "ties":
        g = synth.integer_grid(rows=20, cols=20, seed=9)
    else:
        g = synth.random_sparse(V=600, avg_deg=4, seed=41, directed=True)
    outs, visits = [], []
    for order in (0, 1):
        eng = E.Engine.from_synth(g, layout="csr")
        eng.set_option(E.OPT_SOURCE_ORDER, order)
        eng.set_option(E.OPT_PROFILE, 1)
        eng.set_attached(g.attached)
        A = len(g.attached)
        full = eng.compute_rows(0, A)
        visits.append(eng.stats()["visits"])
        part = eng.compute_rows(A // 3, A - 5)
        eng.close()
        for x, y in zip(full, part):
            assert np.array_equal(x[A // 3:A - 5], y)
        outs.append(full)
    for x, y in zip(*outs):
        assert np.array_equal(x.view(np.uint8) if x.dtype == np.float64 else x,
                              y.view(np.uint8) if y.dtype == np.float64 else y)
    if case == "knn":
        assert visits[1] < 0.6 * visits[0], visits
    st = compare(g, layout="csr")  # default order against the oracle
    assert st["dense"] == 0


@pytest.mark.parametrize("case", ["sparse", "tree_heavy", "vloss_prefer", "int_ties", "chung_lu"])
def test_pendant_tree_pruning_same_results(case):
    """OPT_PRUNE_PENDANT (default): the relaxation view without the pendant trees that hold
    no attached vertex gives bit-identical attached-pair matrices (latency, reliability,
    hops, kind) to the full graph, and the oracle's; full sssp rows still cover every
    vertex"""
    if case == "sparse":
        g = synth.random_sparse(V=500, avg_deg=2.5, seed=61, A=120)
    elif case == "tree_heavy":
        g = synth.random_sparse(V=700, avg_deg=2.1, seed=62, A=90, loops=False)
    elif case == "vloss_prefer":
        rng = np.random.default_rng(8)
        g = synth.random_sparse(V=400, avg_deg=2.5, seed=63, A=100, vloss=np.where(rng.random(400) < 0.5, 0.03, np.nan))
        g.prefer_direct = True
    elif case == "int_ties":
        g = synth.random_sparse(V=450, avg_deg=2.4, seed=64, A=110, int_lat=True)
    else:
        g = synth.chung_lu(V=20_000, A=700)
    mats = []
    for prune in (0, 1):
        eng = E.Engine.from_synth(g, layout="csr")
        eng.set_option(E.OPT_PRUNE_PENDANT, prune)
        eng.set_attached(g.attached)
        mats.append(eng.compute_rows(want_kind=True))
        st = eng.stats()
        assert (st["pruned_vertices"] > 0) == bool(prune), st["pruned_vertices"]
        if prune:
            d, _, _, _ = eng.sssp(np.asarray(g.attached[:3], np.int32))
            assert np.isfinite(d).sum() > 0
        eng.close()
    for x, y in zip(*mats):
        assert np.array_equal(x.view(np.uint8) if x.dtype == np.float64 else x,
                              y.view(np.uint8) if y.dtype == np.float64 else y)
    if case != "chung_lu":
        compare(g, layout="csr")


@pytest.mark.parametrize("case", ["sparse", "directed", "ties", "vloss_prefer", "multigraph"])
def test_device_driven_rounds_same_results(case):
    """OPT_DEVICE_ROUNDS: worklist rounds driven from the device (item counts read back once
    per block of rounds, k_scan_wl / k_relax_wlp) against host-driven rounds (one read-back
    per round) and the oracle, with several batch groups"""
    g = _case(case)
    st1 = compare(g, layout="csr", device_rounds=2, batches_in_flight=2)
    st0 = compare(g, layout="csr", device_rounds=0, batches_in_flight=2)
    assert st1["rounds"] == st0["rounds"] and st1["wl_launches"] == st1["relax_launches"]


@pytest.mark.parametrize("case", ["sparse", "ties", "vloss_prefer", "multigraph"])
def test_csr_device_rounds_heavy_grid_mode(case):
    """Device-driven rounds (OPT_DEVICE_ROUNDS=2) over several batch groups: the persistent
    kernel walks the virtual grid in rounds with at least half the pairs active and the
    worklist otherwise; the same matrices as the oracle's, bit for bit"""
    g = _case(case)
    st = compare(g, layout="csr", device_rounds=2, batches_in_flight=2)
    assert st["dense"] == 0 and st["host_syncs"] < st["rounds"]
