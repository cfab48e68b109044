"""CPU: pin the oracle (the checker) before trusting it.

* against the reference's own data: the shipped topology (direct rule) and the
  1-vertex test topologies of src/test/**/*.test.shadow.config.xml;
* against independent shortest-path implementations (scipy, networkx) for distances;
* igraph-specific semantics restated in topo_oracle.c: get_eid lowest id,
  completeness count, incidence order, self-path rule;
* regression pins (tests/golden/synthetic_*.npz).
"""
import json
import lzma
import os

import networkx as nx
import numpy as np
import pytest
import scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra as sp_dijkstra

from oracle import oracle as O
from oracle.graphml_ref import read_graphml
from shadow_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def og_of(g):
    return O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss, directed=g.directed)


def test_shipped_topology_direct_rule():
    g = read_graphml(lzma.open(os.path.join(GOLD, "c1_topology.graphml.xml.xz"), "rt").read())
    assert (g.n, len(g.src)) == (183, 16836)
    og = O.from_refgraph(g)
    assert og.is_complete()
    gold = np.load(os.path.join(GOLD, "c1_direct.npz"))
    att = np.arange(g.n, dtype=np.int32)
    lat, rel, hops, kind, fails = og.pair_rows(og.flags(), att)
    assert fails == 0
    assert (kind == O.KIND_DIRECT).all() and (hops == 1).all()
    assert np.array_equal(lat, gold["lat"])
    assert np.array_equal(rel, gold["rel"])


def test_reference_test_graphs():
    cases = json.load(open(os.path.join(GOLD, "ref_test_graphs.json")))
    seen = set()
    for c in cases:
        g = read_graphml(c["graphml"])
        og = O.from_refgraph(g)
        assert og.is_complete()  # one vertex + self-loop: 2 incident - 1 >= 1
        lat, rel, hops, kind, _ = og.pair_rows(og.flags(), np.array([0], np.int32))
        assert lat[0, 0] == c["self_latency"] == 50.0
        assert rel[0, 0] == c["self_reliability"]
        seen.add(c["self_reliability"])
    # example config: 0.99 (resource/examples/shadow.config.xml:11-21); lossless / lossy tests
    assert seen == {0.99, 1.0, 0.75}


@pytest.mark.parametrize("seed,directed", [(1, False), (2, False), (3, True), (4, True)])
def test_distances_vs_scipy(seed, directed):
    g = synth.random_sparse(V=400, avg_deg=5, seed=seed, directed=directed)
    og = og_of(g)
    m = g.src != g.dst
    a = sp.coo_matrix((g.latency[m], (g.src[m], g.dst[m])), shape=(g.n, g.n))
    # parallel edges: keep the minimum latency (coo->csr would sum them)
    best = {}
    for s, t, w in zip(a.row, a.col, a.data):
        k = (s, t) if directed else (min(s, t), max(s, t))
        best[k] = min(best.get(k, np.inf), w)
    r, c, w = zip(*[(k[0], k[1], v) for k, v in best.items()])
    csr = sp.csr_matrix((w, (r, c)), shape=(g.n, g.n))
    for s in (0, 17, 123):
        d, _ = og.dijkstra(s)
        ds = sp_dijkstra(csr, directed=directed, indices=s)
        assert np.array_equal(np.where(d < 0, np.inf, d), ds)


def test_distances_vs_networkx_and_paths_are_shortest():
    g = synth.random_sparse(V=200, avg_deg=4, seed=8)
    og = og_of(g)
    G = nx.Graph()
    for s, t, w in zip(g.src, g.dst, g.latency):
        if s != t:
            G.add_edge(int(s), int(t), weight=float(w))
    d, parent = og.dijkstra(5)
    nd = nx.single_source_dijkstra_path_length(G, 5)
    for v, dv in nd.items():
        assert abs(d[v] - dv) <= 1e-9 * max(1.0, dv)
        # the oracle's path latency (left fold, topology.c:1473-1499) equals d(v) exactly
        p = og.path(5, v, parent)
        acc = 0.0
        for a, b in zip(p[:-1], p[1:]):
            acc += g.latency[og.get_eid(a, b)]
        assert acc == d[v]


def test_get_eid_lowest_and_undirected():
    n = 5
    src = np.array([0, 1, 2, 1, 3, 3], np.int32)
    dst = np.array([1, 0, 2, 2, 4, 4], np.int32)
    og = O.OracleGraph(n, src, dst, np.ones(6) * 2, np.zeros(6))
    assert og.get_eid(0, 1) == 0 and og.get_eid(1, 0) == 0  # parallel: lowest id
    assert og.get_eid(2, 2) == 2
    assert og.get_eid(2, 1) == 3
    assert og.get_eid(4, 3) == 4
    assert og.get_eid(0, 4) == -1
    ogd = O.OracleGraph(n, src, dst, np.ones(6) * 2, np.zeros(6), directed=True)
    assert ogd.get_eid(1, 0) == 1 and ogd.get_eid(0, 1) == 0 and ogd.get_eid(2, 1) == -1


def test_completeness_rule():
    # complete simple graph with loops -> complete; remove one loop -> incomplete
    n = 6
    iu, ju = np.triu_indices(n, 0)
    og = O.OracleGraph(n, iu.astype(np.int32), ju.astype(np.int32), np.ones(len(iu)), np.zeros(len(iu)))
    assert og.is_complete()
    keep = ~((iu == 3) & (ju == 3))
    og2 = O.OracleGraph(n, iu[keep].astype(np.int32), ju[keep].astype(np.int32), np.ones(keep.sum()),
                        np.zeros(keep.sum()))
    assert not og2.is_complete()
    # no self loops at all: every vertex has n-1 < n incident edges -> incomplete
    iu1, ju1 = np.triu_indices(n, 1)
    og3 = O.OracleGraph(n, iu1.astype(np.int32), ju1.astype(np.int32), np.ones(len(iu1)), np.zeros(len(iu1)))
    assert not og3.is_complete()


def test_self_path_rule_first_strict_min():
    # vertex 0: edges (0,1) lat 5 loss .1, loop lat 5 loss .3, (0,2) lat 7
    src = np.array([0, 0, 0, 1], np.int32)
    dst = np.array([1, 0, 2, 2], np.int32)
    lat = np.array([5.0, 5.0, 7.0, 1.0])
    loss = np.array([0.1, 0.3, 0.0, 0.0])
    og = O.OracleGraph(3, src, dst, lat, loss)
    l, r = og.self_path(0)
    # incidence order of vertex 0 (igraph_incident OUT, undirected): out part = edges with
    # from==0 (only the loop, stored from=max=0), then in part by neighbour: loop, (0,1), (0,2)
    assert l == 10.0
    assert r == (1 - 0.3) ** 2


def test_heap_pop_order_is_nondecreasing():
    g = synth.random_sparse(V=300, avg_deg=4, seed=31, int_lat=True)
    og = og_of(g)
    d, parent, order = og.dijkstra(0, want_order=True)
    assert np.all(np.diff(d[order]) >= 0)
    assert len(order) == g.n


def test_regression_pins():
    for name in ("synthetic_sparse", "synthetic_ties", "synthetic_directed"):
        z = np.load(os.path.join(GOLD, name + ".npz"))
        og = O.OracleGraph(int(z["n"]), z["src"], z["dst"], z["latency"], z["packetloss"], z["vloss"],
                           directed=bool(z["directed"]))
        lat, rel, hops, kind, _ = og.pair_rows(og.flags(), z["attached"])
        assert np.array_equal(lat, z["lat"]) and np.array_equal(rel, z["rel"])
        assert np.array_equal(hops, z["hops"]) and np.array_equal(kind, z["kind"])


def test_tie_detector_flags_integer_grid():
    g = synth.integer_grid(rows=6, cols=6, seed=1)
    og = og_of(g)
    d, _ = og.dijkstra(0)
    tie = og.tie_vertices(0, d)
    assert tie.sum() > 0
    g2 = synth.random_sparse(V=300, avg_deg=4, seed=2)
    og2 = og_of(g2)
    d2, _ = og2.dijkstra(0)
    assert og2.tie_vertices(0, d2).sum() == 0


@pytest.mark.parametrize("case", ["grid", "grid_big", "int_random", "int_directed", "ties_fixture"])
def test_tie_break_second_restatement(case):
    """The parity-unpinned branch has no reference fixture (igraph is absent), so the
    tie-broken predecessors of topo_oracle.c are cross-checked against a second, independent
    restatement of igraph's heap Dijkstra in pure Python (oracle/igraph_heap_ref.py), on
    integer-latency graphs where heap-order ties are everywhere: parent edges, distances and
    the pair rows must agree exactly."""
    from oracle.igraph_heap_ref import RefGraph
    if case == "grid":
        g = synth.integer_grid(rows=8, cols=9, seed=3)
    elif case == "grid_big":
        g = synth.integer_grid(rows=14, cols=14, seed=11, max_lat=2)
    elif case == "int_random":
        g = synth.random_sparse(V=150, avg_deg=5, seed=33, int_lat=True)
    elif case == "int_directed":
        g = synth.random_sparse(V=120, avg_deg=4, seed=34, int_lat=True, directed=True)
    else:
        d = np.load(os.path.join(GOLD, "synthetic_ties.npz"))
        g = synth.SynthGraph("ties", int(d["n"]), d["src"], d["dst"], d["latency"], d["packetloss"], d["vloss"],
                             d["attached"], directed=bool(d["directed"]))
    og = og_of(g)
    rg = RefGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss, directed=g.directed)
    att = np.asarray(g.attached)
    lat, rel, hops, kind, _ = og.pair_rows(og.flags(), att)
    ties = 0
    for i, s in enumerate(att[: min(len(att), 24)]):
        d_c, p_c = og.dijkstra(int(s), targets=att)
        d_p, p_p = rg.dijkstra(int(s), att)
        assert np.array_equal(np.asarray(d_p), d_c)
        assert np.array_equal(np.asarray(p_p), p_c), f"source {s}: parent edges differ"
        ties += int(og.tie_vertices(int(s), d_c).sum())
        for j, t in enumerate(att):
            if kind[i, j] != O.KIND_DIJKSTRA:
                continue
            pl, pr, ph = rg.pair(int(s), int(t), p_p)
            assert (pl, pr, ph) == (lat[i, j], rel[i, j], hops[i, j]), (s, t)
    assert ties > 0  # the fixtures do exercise heap-order ties


def test_path_cache_model_reference_quirks():
    """oracle/path_cache_ref.py restates topology.c's cache literally: in an undirected graph
    the second direction of a pair is served by the first one's Path; in a directed graph
    _topology_shouldStorePath refuses (s, t) once (t, s) is cached (topology.c:1311-1317), so
    the query (s, t) misses, reruns s's Dijkstra on every call and is answered with the (t, s)
    Path by the post-computation fallback (topology.c:2033-2038)"""
    import numpy as np
    from oracle.path_cache_ref import RefPathCache
    lat = np.array([[2.0, 5.0, 7.0], [6.0, 2.0, 4.0], [7.5, 4.5, 3.0]])
    kind = np.array([[2, 3, 3], [3, 2, 3], [3, 3, 2]])
    adj = lambda i, j: False  # noqa: E731
    und = RefPathCache(lat, kind, directed=False, complete=False, prefer_direct=False, adjacent=adj)
    assert und.get_path_entry(1, 0) == (1, 0)
    assert und.get_path_entry(0, 1) == (1, 0)  # served by the reverse Path
    assert und.get_path_entry(0, 2) == (0, 2)  # source 0's Dijkstra: its own row
    # source 1's run stored (1,0)=6 and (1,2)=4, not (1,1): igraph's path to the source itself
    # is [] (topology.c:1815); source 0's run stored nothing lower
    assert und.dijkstra_runs == 2 and und.upcalls == [6.0, 4.0] and und.min_latency == 4.0
    assert (0, 0) not in und.cache and (1, 1) not in und.cache
    assert und.get_path_entry(0, 0) == (0, 0) and und.self_paths == 1  # a self-path run
    assert und.upcalls == [6.0, 4.0, 2.0]
    assert und.get_path_entry(0, 0) == (0, 0) and und.self_paths == 1  # now a hit
    # the [s]-path igraph (self_loop_rule): the run stores the source's self-loop path (the
    # diagonal); a query (s, s) that comes first caches the self-path rule's value instead,
    # and a source without a self-loop fails its Dijkstra run (after storing the rest)
    slat, skind = np.array([9.0, 8.0, 7.0]), np.array([2, 2, 2])
    lk = kind.copy()
    lk[2, 2] = 0  # vertex 2 has no self-loop
    sl = RefPathCache(lat, lk, directed=False, complete=False, prefer_direct=False, adjacent=adj,
                      self_loop_rule=True, self_lat=slat, self_kind=skind)
    assert sl.get_path_entry(0, 0) == (0, 0) and 0 in sl.self_claimed and sl.cache[(0, 0)] == 9.0
    assert sl.get_path_entry(1, 2) == (1, 2) and (1, 1) in sl.cache and 1 not in sl.self_claimed
    assert sl.cache[(1, 1)] == 2.0  # the [s] path's value
    assert sl.get_path_entry(2, 0) is None and (2, 0) in sl.cache  # stored, but the run failed
    assert sl.get_path_entry(2, 0) == (2, 0)  # a hit afterwards
    d = RefPathCache(lat, kind, directed=True, complete=False, prefer_direct=False, adjacent=adj)
    assert d.get_path_entry(1, 0) == (1, 0) and d.dijkstra_runs == 1
    assert d.get_path_entry(0, 1) == (1, 0) and d.dijkstra_runs == 2  # the reverse Path
    assert d.get_path_entry(0, 1) == (1, 0) and d.dijkstra_runs == 3  # a miss every time
    assert d.get_path_entry(0, 2) == (0, 2) and (0, 1) not in d.cache  # stored by run 2
    assert d.get_path_entry(0, 2) == (0, 2) and d.dijkstra_runs == 3  # a hit
