"""Shared helpers: run the HIP engine and the CPU oracle on the same graph and compare."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from shadow_amd import engine as E


def oracle_for(g):
    return O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss, directed=g.directed)


def oracle_matrix(g, self_loop_rule=False, nthreads=4):
    og = oracle_for(g)
    flags = og.flags(prefer_direct=g.prefer_direct, self_dijkstra_loop=self_loop_rule)
    lat, rel, hops, kind, _ = og.pair_rows(flags, g.attached, nthreads=nthreads)
    return lat, rel, hops, kind, og


def engine_matrix(g, self_loop_rule=False, layout="auto", **opts):
    eng = E.Engine.from_synth(g, self_dijkstra_loop=self_loop_rule, layout=layout)
    for k, v in opts.items():
        eng.set_option(getattr(E, "OPT_" + k.upper()), v)
    eng.set_attached(g.attached)
    lat, rel, hops, kind = eng.compute_rows()
    st = eng.stats()
    eng.close()
    return lat, rel, hops, kind, st


def assert_bitexact(name, got, want):
    if got.dtype.kind == "f":
        same = (got.view(np.uint64) == want.view(np.uint64))
    else:
        same = got == want
    if not same.all():
        bad = np.argwhere(~same)
        i, j = bad[0]
        raise AssertionError(f"{name}: {len(bad)} mismatches, first at {tuple(bad[0])}: got {got[i, j]!r} "
                             f"want {want[i, j]!r}")


def compare(g, self_loop_rule=False, rel_tol=0.0, layout="auto", **opts):
    lat_o, rel_o, hops_o, kind_o, _ = oracle_matrix(g, self_loop_rule)
    lat_e, rel_e, hops_e, kind_e, st = engine_matrix(g, self_loop_rule, layout=layout, **opts)
    assert_bitexact("kind", kind_e, kind_o)
    assert_bitexact("latency", lat_e, lat_o)
    assert_bitexact("hops", hops_e, hops_o)
    if rel_tol == 0.0:
        assert_bitexact("reliability", rel_e, rel_o)
    else:
        np.testing.assert_allclose(rel_e, rel_o, rtol=rel_tol, atol=0)
    return st
