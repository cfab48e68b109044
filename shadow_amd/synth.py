"""Synthetic topologies for the BASELINE.json configs.

Every generator returns a :class:`SynthGraph` in the reference's vocabulary: an
undirected GraphML-style edge list (edge index = GraphML <edge> order), per-edge
``latency`` (ms, f64, full random mantissa) and ``packetloss``, per-vertex
``packetloss`` (0.0 unless stated), a self-loop on every vertex as in atlas-style
Shadow topologies, one strongly connected component (required by
/root/reference/src/main/routing/topology.c:800-806), and the attached vertex set
(the unique vertices hosts are attached to, topology.c:2384).

Seeds are fixed per config as SURVEY.md section 8d lists them.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class SynthGraph:
    name: str
    n: int
    src: np.ndarray          # int32 [E]
    dst: np.ndarray          # int32 [E]
    latency: np.ndarray      # float64 [E] ms
    packetloss: np.ndarray   # float64 [E]
    vertex_packetloss: np.ndarray  # float64 [V] (NaN = attribute absent)
    attached: np.ndarray     # int32 [A] unique attached vertices
    directed: bool = False
    prefer_direct: bool = False
    meta: dict = field(default_factory=dict)

    @property
    def m(self):
        return len(self.src)

    @property
    def n_arcs(self):
        """non-loop arcs of the SSSP in-CSR (2 per undirected non-loop edge)"""
        nl = int(np.count_nonzero(self.src != self.dst))
        return nl if self.directed else 2 * nl


def _loops(n, rng, lo, hi):
    v = np.arange(n, dtype=np.int32)
    return v, v, rng.uniform(lo, hi, n)


def _components(n, src, dst):
    """connected components (undirected) with scipy"""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import connected_components
    a = sp.coo_matrix((np.ones(len(src), np.int8), (src, dst)), shape=(n, n))
    return connected_components(a, directed=False)


def _giant(n, src, dst, *arrays):
    ncomp, lab = _components(n, src, dst)
    if ncomp == 1:
        return n, src, dst, arrays
    big = np.bincount(lab).argmax()
    keep_v = lab == big
    remap = -np.ones(n, np.int64)
    remap[keep_v] = np.arange(int(keep_v.sum()))
    keep_e = keep_v[src] & keep_v[dst]
    return (int(keep_v.sum()), remap[src[keep_e]].astype(np.int32), remap[dst[keep_e]].astype(np.int32),
            tuple(a[keep_e] for a in arrays))


def _finish(name, n, src, dst, lat, loss, attached, **meta):
    return SynthGraph(name=name, n=n, src=np.ascontiguousarray(src, np.int32),
                      dst=np.ascontiguousarray(dst, np.int32),
                      latency=np.ascontiguousarray(lat, np.float64),
                      packetloss=np.ascontiguousarray(loss, np.float64),
                      vertex_packetloss=np.zeros(n, np.float64),
                      attached=np.ascontiguousarray(attached, np.int32), meta=meta)


def geometric_complete_ish(V=10_000, A=1_000, drop=0.05, seeds=(1, 2, 3)):
    """C2: points uniform in the unit square (seed 1), latency = 1 + 200*dist + U[0,1e-3],
    each non-loop pair dropped with p=0.05 (seed 2) so the graph is incomplete, A distinct
    attached vertices (seed 3)."""
    r1 = np.random.default_rng(seeds[0])
    pts = r1.random((V, 2))
    iu, ju = np.triu_indices(V, 1)
    iu = iu.astype(np.int32)
    ju = ju.astype(np.int32)
    r2 = np.random.default_rng(seeds[1])
    keep = r2.random(len(iu)) >= drop
    iu, ju = iu[keep], ju[keep]
    d = np.sqrt(((pts[iu] - pts[ju]) ** 2).sum(1))
    lat = 1.0 + 200.0 * d + r1.uniform(0.0, 1e-3, len(iu))
    loss = r1.uniform(0.0, 0.02, len(iu))
    lv, lu, llat = _loops(V, r1, 1.0, 1.001)
    src = np.concatenate([lv, iu])
    dst = np.concatenate([lu, ju])
    lat = np.concatenate([llat, lat])
    loss = np.concatenate([r1.uniform(0.0, 0.02, V), loss])
    r3 = np.random.default_rng(seeds[2])
    att = np.sort(r3.choice(V, size=min(A, V), replace=False))
    return _finish("C2-geometric", V, src, dst, lat, loss, att, drop=drop)


def knn_geographic(V=7_000, k=16, A=None, seed=4):
    """C3 (Tor stand-in): geographic k-NN graph (k=16) on the unit square, latency =
    1 + 200*dist + U[0,1e-3], giant component, every vertex attached by default."""
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    pts = rng.random((V, 2))
    _, nb = cKDTree(pts).query(pts, k=k + 1)
    a = np.repeat(np.arange(V), k)
    b = nb[:, 1:].reshape(-1)
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    pairs = np.unique(lo.astype(np.int64) * V + hi)
    iu = (pairs // V).astype(np.int32)
    ju = (pairs % V).astype(np.int32)
    d = np.sqrt(((pts[iu] - pts[ju]) ** 2).sum(1))
    lat = 1.0 + 200.0 * d + rng.uniform(0.0, 1e-3, len(iu))
    loss = rng.uniform(0.0, 0.02, len(iu))
    n, iu, ju, (lat, loss) = _giant(V, iu, ju, lat, loss)
    lv, lu, llat = _loops(n, rng, 1.0, 1.001)
    src = np.concatenate([lv, iu])
    dst = np.concatenate([lu, ju])
    att = np.arange(n, dtype=np.int32) if A is None else np.sort(rng.choice(n, size=min(A, n), replace=False))
    return _finish("C3-knn", n, src, dst, np.concatenate([llat, lat]),
                   np.concatenate([rng.uniform(0.0, 0.02, n), loss]), att, k=k)


def barabasi_albert(V=100_000, m=3, A=10_000, seeds=(5, 6)):
    """C4: Barabasi-Albert m=3 (seed 5), lognormal latency (median 20 ms, sigma 1),
    A attached vertices (seed 6)."""
    rng = np.random.default_rng(seeds[0])
    src = np.empty((V - m) * m, np.int32)
    dst = np.empty((V - m) * m, np.int32)
    rep = np.empty(2 * (V - m) * m + m, np.int64)
    rep[:m] = np.arange(m)
    nrep = m
    k = 0
    targets = np.arange(m)
    for v in range(m, V):
        src[k:k + m] = v
        dst[k:k + m] = targets
        k += m
        rep[nrep:nrep + m] = targets
        rep[nrep + m:nrep + 2 * m] = v
        nrep += 2 * m
        # m distinct targets proportional to degree
        t = set()
        while len(t) < m:
            t.update(rep[rng.integers(0, nrep, m - len(t))].tolist())
        targets = np.fromiter(t, np.int64, m)
    lat = 20.0 * np.exp(rng.standard_normal(len(src)))
    loss = rng.uniform(0.0, 0.02, len(src))
    lv, lu, llat = _loops(V, rng, 0.5, 1.5)
    r2 = np.random.default_rng(seeds[1])
    att = np.sort(r2.choice(V, size=min(A, V), replace=False))
    return _finish("C4-ba", V, np.concatenate([lv, src]), np.concatenate([lu, dst]),
                   np.concatenate([llat, lat]), np.concatenate([rng.uniform(0.0, 0.02, V), loss]), att, m=m)


def chung_lu(V=1_000_000, mean_degree=4.0, gamma=2.5, A=50_000, seeds=(7, 8)):
    """C5: Chung-Lu power-law graph (exponent gamma), mean degree 4 (seed 7), giant
    component, lognormal latency, A attached vertices (seed 8)."""
    rng = np.random.default_rng(seeds[0])
    i = np.arange(1, V + 1, dtype=np.float64)
    w = i ** (-1.0 / (gamma - 1.0))
    w *= mean_degree * V / w.sum()
    p = w / w.sum()
    m = int(mean_degree * V / 2)
    a = rng.choice(V, size=m, p=p)
    b = rng.choice(V, size=m, p=p)
    ok = a != b
    lo, hi = np.minimum(a[ok], b[ok]), np.maximum(a[ok], b[ok])
    pairs = np.unique(lo.astype(np.int64) * V + hi)
    rng.shuffle(pairs)
    iu = (pairs // V).astype(np.int32)
    ju = (pairs % V).astype(np.int32)
    lat = 10.0 * np.exp(0.75 * rng.standard_normal(len(iu)))
    loss = rng.uniform(0.0, 0.02, len(iu))
    n, iu, ju, (lat, loss) = _giant(V, iu, ju, lat, loss)
    lv, lu, llat = _loops(n, rng, 0.5, 1.5)
    r2 = np.random.default_rng(seeds[1])
    att = np.sort(r2.choice(n, size=min(A, n), replace=False))
    return _finish("C5-chunglu", n, np.concatenate([lv, iu]), np.concatenate([lu, ju]),
                   np.concatenate([llat, lat]), np.concatenate([rng.uniform(0.0, 0.02, n), loss]), att,
                   gamma=gamma)


def with_vertex_loss(g: SynthGraph, frac=0.3, hi=0.02, seed=9) -> SynthGraph:
    """The same graph with a vertex `packetloss` attribute on a `frac` share of the vertices,
    U[0, hi] (seed 9); the rest leave it absent (NaN).  Targets with vertex loss take the
    reference's full path fold (topology.c:1429-1462), the C4 vertex-loss variant ("C4L")."""
    import copy
    rng = np.random.default_rng(seed)
    out = copy.copy(g)
    out.vertex_packetloss = np.where(rng.random(g.n) < frac, rng.uniform(0.0, hi, g.n), np.nan)
    out.name = g.name + "+vloss"
    return out


def integer_grid(rows=20, cols=20, seed=11, max_lat=3, A=None):
    """Tie-stress: grid with small integer latencies, so many vertices have several
    shortest-path predecessors at identical distance (heap-order ties)."""
    rng = np.random.default_rng(seed)
    idx = np.arange(rows * cols).reshape(rows, cols)
    h = np.stack([idx[:, :-1].ravel(), idx[:, 1:].ravel()], 1)
    v = np.stack([idx[:-1, :].ravel(), idx[1:, :].ravel()], 1)
    e = np.concatenate([h, v])
    n = rows * cols
    lat = rng.integers(1, max_lat + 1, len(e)).astype(np.float64)
    loss = rng.integers(0, 5, len(e)) / 100.0
    att = np.arange(n, dtype=np.int32) if A is None else np.sort(rng.choice(n, size=A, replace=False))
    g = _finish("tie-grid", n, e[:, 0], e[:, 1], lat, loss, att)
    return g


def random_sparse(V=500, avg_deg=4.0, seed=21, A=None, directed=False, loops=True, vloss=None,
                  int_lat=False):
    """Small random connected graph for parity tests (spanning tree + extra edges)."""
    rng = np.random.default_rng(seed)
    parent = np.array([rng.integers(0, i) for i in range(1, V)], np.int32)
    child = np.arange(1, V, dtype=np.int32)
    extra = int(max(0, avg_deg * V / 2 - (V - 1)))
    a = rng.integers(0, V, extra).astype(np.int32)
    b = rng.integers(0, V, extra).astype(np.int32)
    ok = a != b
    src = np.concatenate([parent, a[ok]])
    dst = np.concatenate([child, b[ok]])
    lo, hi = np.minimum(src, dst), np.maximum(src, dst)
    _, first = np.unique(lo.astype(np.int64) * V + hi, return_index=True)
    first.sort()
    src, dst = src[first], dst[first]
    if directed:
        # add reverse arcs so the graph is strongly connected
        src, dst = np.concatenate([src, dst]), np.concatenate([dst, src])
        perm = rng.permutation(len(src))
        src, dst = src[perm], dst[perm]
    if int_lat:
        lat = rng.integers(1, 6, len(src)).astype(np.float64)
    else:
        lat = 20.0 * np.exp(rng.standard_normal(len(src)))
    loss = rng.uniform(0.0, 0.05, len(src))
    if loops:
        lv = np.arange(V, dtype=np.int32)
        src = np.concatenate([lv, src])
        dst = np.concatenate([lv, dst])
        lat = np.concatenate([rng.uniform(0.5, 3.0, V) if not int_lat else rng.integers(1, 4, V).astype(float), lat])
        loss = np.concatenate([rng.uniform(0.0, 0.05, V), loss])
    att = np.arange(V, dtype=np.int32) if A is None else np.sort(rng.choice(V, size=A, replace=False))
    g = _finish("random-sparse", V, src, dst, lat, loss, att)
    g.directed = directed
    if vloss is not None:
        g.vertex_packetloss = np.asarray(vloss, np.float64)
    return g


CONFIGS = {
    "C2": lambda scale=1.0: geometric_complete_ish(V=int(10_000 * scale), A=max(8, int(1_000 * scale))),
    "C3": lambda scale=1.0: knn_geographic(V=int(7_000 * scale)),
    "C4": lambda scale=1.0: barabasi_albert(V=int(100_000 * scale), A=max(8, int(10_000 * scale))),
    "C5": lambda scale=1.0: chung_lu(V=int(1_000_000 * scale), A=max(8, int(50_000 * scale))),
}


def to_graphml(g: SynthGraph, bandwidth=(10240, 10240), prefer_direct=None, extra_vattr=None) -> str:
    """Serialise as Shadow-style GraphML (same key layout as the shipped topology)."""
    out = ['<?xml version="1.0" encoding="utf-8"?>'
           '<graphml xmlns="http://graphml.graphdrawing.org/xmlns">',
           '  <key attr.name="packetloss" attr.type="double" for="edge" id="d9" />',
           '  <key attr.name="latency" attr.type="double" for="edge" id="d7" />',
           '  <key attr.name="bandwidthup" attr.type="int" for="node" id="d4" />',
           '  <key attr.name="bandwidthdown" attr.type="int" for="node" id="d3" />',
           '  <key attr.name="packetloss" attr.type="double" for="node" id="d0" />']
    if extra_vattr:
        for name, (kid, typ, _) in extra_vattr.items():
            out.append(f'  <key attr.name="{name}" attr.type="{typ}" for="node" id="{kid}" />')
    if prefer_direct is not None:
        out.append('  <key attr.name="preferdirectpaths" attr.type="string" for="graph" id="g0" />')
    out.append(f'  <graph edgedefault="{"directed" if g.directed else "undirected"}">')
    if prefer_direct is not None:
        out.append(f'    <data key="g0">{prefer_direct}</data>')
    for v in range(g.n):
        vl = g.vertex_packetloss[v]
        line = f'    <node id="v{v}"><data key="d3">{bandwidth[0]}</data><data key="d4">{bandwidth[1]}</data>'
        if not np.isnan(vl):
            line += f'<data key="d0">{float(vl)!r}</data>'
        if extra_vattr:
            for name, (kid, typ, vals) in extra_vattr.items():
                if vals[v] is not None:
                    line += f'<data key="{kid}">{vals[v]}</data>'
        out.append(line + '</node>')
    for e in range(g.m):
        out.append(f'    <edge source="v{g.src[e]}" target="v{g.dst[e]}"><data key="d7">{float(g.latency[e])!r}</data>'
                   f'<data key="d9">{float(g.packetloss[e])!r}</data></edge>')
    out.append('  </graph>\n</graphml>\n')
    return "\n".join(out)
