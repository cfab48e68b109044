"""Full-size parity on BASELINE.json's configs C2-C5 (SURVEY.md 8d generators, fixed seeds).

The engine computes whole attached rows at the real graph size (C2: every one of the 1000
sources, i.e. the bench workload itself; C3-C5: a source block spanning several batches).
The north-star matrix (C4: all 10^4 x 10^4 attached pairs) and the whole C3 matrix
(7000 x 7000) are compared with the CPU oracle bit for bit, every pair; C2 and C5 one full
64-source batch each, every row of it (the oracle over the box's CPU share: the C4 matrix
is ~25 s of heap-exact Dijkstra on 16 threads).  Every computed row is also checked for
size-independent properties: the reference's pair kinds, hop/latency consistency, and
d(s, t) <= w(s, t) wherever the arc exists (a shortest path is never longer than the edge).
"""
import os

import numpy as np
import pytest

from paritylib import assert_bitexact, oracle_for
from shadow_amd import engine as E
from shadow_amd import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

KIND_DIJKSTRA = 3


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or n))


def _run(g, r0, r1, sample, block=None, **opts):
    """engine rows [r0, r1); the oracle's rows `sample` one by one, and the row block
    `block` = (b0, b1) in one multi-threaded oracle call, compared bit for bit"""
    eng = E.Engine.from_synth(g)
    for k, v in opts.items():
        eng.set_option(getattr(E, "OPT_" + k.upper()), v)
    eng.set_attached(g.attached)
    lat, rel, hops, kind = eng.compute_rows(r0, r1)
    st = eng.stats()
    eng.close()
    og = oracle_for(g)
    flags = og.flags(prefer_direct=g.prefer_direct)
    for r in sample:
        olat, orel, ohops, okind, _ = og.pair_rows(flags, g.attached, r, r + 1, nthreads=1)
        i = r - r0
        assert_bitexact(f"kind row {r}", kind[i:i + 1], okind)
        assert_bitexact(f"latency row {r}", lat[i:i + 1], olat)
        assert_bitexact(f"hops row {r}", hops[i:i + 1], ohops)
        assert_bitexact(f"reliability row {r}", rel[i:i + 1], orel)
    if block is not None:
        b0, b1 = block
        olat, orel, ohops, okind, fails = og.pair_rows(flags, g.attached, b0, b1, nthreads=_threads())
        sl = slice(b0 - r0, b1 - r0)
        assert_bitexact(f"kind rows [{b0},{b1})", kind[sl], okind)
        assert_bitexact(f"latency rows [{b0},{b1})", lat[sl], olat)
        assert_bitexact(f"hops rows [{b0},{b1})", hops[sl], ohops)
        assert_bitexact(f"reliability rows [{b0},{b1})", rel[sl], orel)
        del olat, orel, ohops, okind
    og.close()
    # properties of every computed row
    dj = kind == KIND_DIJKSTRA
    assert dj.any()
    assert (lat[dj] > 0).all() and (hops[dj] >= 1).all()
    assert ((rel[dj] > 0) & (rel[dj] <= 1)).all()
    assert (lat[kind == 0] == -1).all()
    # shortest path <= the direct arc: check against the edge list
    A = len(g.attached)
    pos = np.full(g.n, -1, np.int64)
    pos[g.attached] = np.arange(A)
    src, dst = g.src.astype(np.int64), g.dst.astype(np.int64)
    for a, b in ((src, dst), (dst, src)):
        pa, pb = pos[a], pos[b]
        keep = (pa >= r0) & (pa < r1) & (pb >= 0) & (a != b)
        i, j = pa[keep] - r0, pb[keep]
        w = g.latency[keep]
        ok = (kind[i, j] != KIND_DIJKSTRA) | (lat[i, j] <= w)
        assert ok.all(), f"{(~ok).sum()} pairs longer than their direct arc"
    return st


def test_c2_geometric_full_matrix():
    """The bench workload: V=10^4 complete-ish graph, all 1000 attached sources (16 batches)."""
    g = synth.geometric_complete_ish(V=10_000, A=1_000)
    st = _run(g, 0, 1000, sample=[0, 63, 64, 517, 999])
    assert st["dense"] == 1 and st["replayed_sources"] == 0


def test_c2_pruned_equals_unpruned_full_matrix():
    """The whole 1000x1000 bench matrix from the pruned sweep (default) and from the
    unpruned one, bit for bit: every pair of the headline workload, not a sample."""
    g = synth.geometric_complete_ish(V=10_000, A=1_000)
    mats = []
    for prune in (1, 0):
        eng = E.Engine.from_synth(g)
        eng.set_option(E.OPT_DENSE_PRUNE, prune)
        eng.set_attached(g.attached)
        mats.append(eng.compute_rows())
        eng.close()
    for name, x, y in zip(("latency", "reliability", "hops", "kind"), *mats):
        assert_bitexact(name, x, y)


def test_c2_geometric_f64_kernels():
    g = synth.geometric_complete_ish(V=10_000, A=1_000)
    st = _run(g, 0, 192, sample=[5, 130], dense_variant=E.DENSE_F64)
    assert st["dense"] == 1


def test_c2_one_full_batch_vs_oracle():
    """every pair of the first 64-source batch of the bench workload against the oracle"""
    g = synth.geometric_complete_ish(V=10_000, A=1_000)
    _run(g, 0, 64, sample=[], block=(0, 64))


def test_c3_knn_whole_matrix_vs_oracle():
    """C3 (Tor stand-in, 7000 attached vertices): the whole 7000 x 7000 matrix, bit for bit"""
    g = synth.knn_geographic(V=7_000)
    A = len(g.attached)
    _run(g, 0, A, sample=[], block=(0, A))


def test_c4_north_star_whole_matrix_vs_oracle():
    """The north-star workload (BASELINE.json configs[3]): all 10^4 x 10^4 attached pairs of
    the 10^5-vertex Barabasi-Albert graph, bit for bit against the oracle"""
    g = synth.barabasi_albert(V=100_000, A=10_000)
    A = len(g.attached)
    _run(g, 0, A, sample=[], block=(0, A))


def test_c5_chung_lu_full_size():
    """C5: a 128-row block spanning two batches; its first whole batch against the oracle"""
    g = synth.chung_lu(V=1_000_000, A=50_000)
    _run(g, 20_000, 20_128, sample=[20_101], block=(20_000, 20_064))
