"""Full-size parity on BASELINE.json's configs C2-C5 (SURVEY.md 8d generators, fixed seeds).

The engine computes the bench's own workloads at the real graph size.  The north-star
matrix (C4: all 10^4 x 10^4 attached pairs) and the whole C3 matrix (7000 x 7000) are
compared with the CPU oracle bit for bit, every pair (the oracle over the box's CPU share:
the C4 matrix is ~25 s of heap-exact Dijkstra on 16 threads), and so is the whole C2 matrix
(1000 x 1000, the headline workload), and the north-star matrix with vertex loss on 30 % of
the vertices (C4L); C5 (all 50 000 rows in one call, the bench's batch groups) with 64 rows
of every group and the last 64.  Every computed row is
also checked for size-independent properties: the reference's pair kinds, hop/latency
consistency, and d(s, t) <= w(s, t) wherever the arc exists (a shortest path is never
longer than the edge); C5's whole matrix also for d(s, t) = d(t, s) to rounding.
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


def test_c2_r06_step_options_full_matrix():
    """The whole 1000x1000 bench matrix with r06's step defaults (round 0's exact pass leaving
    the untainted seed winners unread, fp16 delta slabs) and without either, bit for bit
    (the defaults are checked against the oracle in test_c2_whole_matrix_vs_oracle)"""
    g = synth.geometric_complete_ish(V=10_000, A=1_000)
    mats = []
    for skip, w16 in ((1, 1), (0, 0), (1, 0), (0, 1)):
        eng = E.Engine.from_synth(g)
        eng.set_option(E.OPT_SEED_SKIP, skip)
        eng.set_option(E.OPT_DELTA_W16, w16)
        eng.set_attached(g.attached)
        mats.append(eng.compute_rows())
        eng.close()
    for other in mats[1:]:
        for name, x, y in zip(("latency", "reliability", "hops", "kind"), mats[0], other):
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


def test_c4_vertex_loss_whole_matrix_vs_oracle():
    """The north-star workload with vertex loss on 30 % of the vertices (U[0, 0.02], the
    bench's C4L variant): every pair whose target carries loss takes the reference's full
    path fold (topology.c:1429-1462, compose's bounded path walk); all 10^4 x 10^4 pairs bit
    for bit against the oracle"""
    g = synth.with_vertex_loss(synth.barabasi_albert(V=100_000, A=10_000))
    A = len(g.attached)
    assert 0.25 < np.mean(~np.isnan(g.vertex_packetloss[g.attached])) < 0.35
    _run(g, 0, A, sample=[], block=(0, A))


def _oracle_rows_check(g, rows, lat, rel, hops, kind):
    """the oracle's rows `rows` (one OpenMP call over the list) against the engine's rows,
    given as host arrays whose row q is matrix row rows[q]"""
    og = oracle_for(g)
    flags = og.flags(prefer_direct=g.prefer_direct)
    olat, orel, ohops, okind, _ = og.pair_rows_list(flags, g.attached, rows, nthreads=_threads())
    og.close()
    assert_bitexact("kind", kind, okind)
    assert_bitexact("latency", lat, olat)
    assert_bitexact("hops", hops, ohops)
    assert_bitexact("reliability", rel, orel)


def test_c2_whole_matrix_vs_oracle():
    """The bench workload with the bench's defaults (all 1000 sources, 16 batches in locality
    order; the sweep in two parts of 9 and 7 batches on two streams, each part's
    read-back-free delta rounds chained on its stream): the whole 1000 x 1000 matrix against
    the oracle, every pair bit for bit (~75 s of oracle over the box's 16 threads)"""
    g = synth.geometric_complete_ish(V=10_000, A=1_000)
    eng = E.Engine.from_synth(g)
    eng.set_attached(g.attached)
    lat, rel, hops, kind = eng.compute_rows()
    st = eng.stats()
    eng.close()
    assert st["dense"] == 1 and st["batches"] == 16
    assert st["full_sweeps"] == 1 and st["delta_sweeps"] >= 2
    rows = np.arange(1000, dtype=np.int32)
    _oracle_rows_check(g, rows, lat, rel, hops, kind)


def test_c2_packed_rows_round_trip():
    """the bench's packed row exchange at C2's full size: the whole 1000 x 1000 block (the
    N-rank runs pack the same rows against 1000 N targets) packed on one engine and
    unpacked on a second one, bit-identical to the computed rows, at under 1/8 of the raw
    20 bytes per pair"""
    import torch
    g = synth.geometric_complete_ish(V=10_000, A=1_000)
    engs = [E.Engine.from_synth(g) for _ in range(2)]
    for e in engs:
        e.set_attached(g.attached)
    A = 1000
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    lat = torch.empty((A, A), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    hops = torch.empty((A, A), dtype=torch.int32, device=dev)
    engs[0].compute_rows_device(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=s)
    cap = E.Engine.packed_capacity(A, A)
    buf = torch.empty(cap, dtype=torch.uint8, device=dev)
    nbytes = engs[0].pack_rows(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), buf.data_ptr(), cap, stream=s)
    out = [torch.empty_like(lat), torch.empty_like(rel), torch.empty_like(hops)]
    engs[1].unpack_rows(0, A, buf.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), stream=s)
    torch.cuda.synchronize(dev)
    for e in engs:
        e.close()
    assert torch.equal(out[0].view(torch.int64), lat.view(torch.int64))
    assert torch.equal(out[1].view(torch.int64), rel.view(torch.int64))
    assert torch.equal(out[2], hops)
    assert nbytes * 8 < A * A * 20, nbytes


def test_c5_whole_matrix_on_device():
    """C5 exactly as the bench times it: all 50 000 rows in one call with the default grouping
    (batch groups sized by HBM, the pools reused across them, grids past 2^24 blocks going
    2-D), the 50 GB of rows left on the device.  Every row is checked there for the
    size-independent properties (kinds, hop / latency / reliability ranges, d(s, t) = d(t, s)
    to rounding in this undirected graph, d(s, t) <= w(s, t) over every attached arc), and 64
    rows of every group plus the last 64 rows against the oracle bit for bit."""
    torch = pytest.importorskip("torch")
    g = synth.chung_lu(V=1_000_000, A=50_000)
    A = len(g.attached)
    dev = torch.device("cuda:0")
    lat = torch.empty((A, A), dtype=torch.float64, device=dev)
    rel = torch.empty((A, A), dtype=torch.float64, device=dev)
    hops = torch.empty((A, A), dtype=torch.int32, device=dev)
    kind = torch.empty((A, A), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    eng = E.Engine.from_synth(g)
    eng.set_attached(g.attached)
    eng.compute_rows_device(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), kind.data_ptr())
    st = eng.stats()
    eng.close()
    assert st["sources"] == A and st["batches"] == (A + 63) // 64
    assert st["groups"] >= 2, "expected several batch groups"
    nb = st["group_batches"]
    # every row, on the device, in blocks of 5000 rows
    diag = torch.arange(A, device=dev)
    assert (kind[diag, diag] == 2).all()  # the self rule on the diagonal
    for r0 in range(0, A, 5000):
        r1 = min(A, r0 + 5000)
        k, l_, h, r = kind[r0:r1], lat[r0:r1], hops[r0:r1], rel[r0:r1]
        dj = k == KIND_DIJKSTRA
        assert int((k == 0).sum()) == 0  # the giant component: every pair routable
        assert bool((l_[dj] > 0).all()) and bool((h[dj] >= 1).all())
        assert bool(((r[dj] > 0) & (r[dj] <= 1)).all())
        lt = lat[:, r0:r1].t()
        rel_err = ((l_ - lt).abs() / torch.maximum(l_, lt))[dj & (kind[:, r0:r1].t() == KIND_DIJKSTRA)]
        assert float(rel_err.max()) <= 1e-12  # the same shortest distance from both ends
        del k, l_, h, r, dj, lt, rel_err
    pos = np.full(g.n, -1, np.int64)
    pos[g.attached] = np.arange(A)
    pa, pb = pos[g.src], pos[g.dst]
    keep = (pa >= 0) & (pb >= 0) & (g.src != g.dst)
    ia = torch.as_tensor(pa[keep], device=dev)
    ib = torch.as_tensor(pb[keep], device=dev)
    w = torch.as_tensor(g.latency[keep], device=dev)
    for x, y in ((ia, ib), (ib, ia)):
        assert bool(((kind[x, y] != KIND_DIJKSTRA) | (lat[x, y] <= w)).all())
    # the oracle: 64 rows spread over every batch group's row range (a batch's worth per
    # group; which rows share a batch follows the engine's locality order), and the last 64
    # rows, the short last batch's range (~450 rows, ~20 s of oracle over 16 threads)
    G = nb * 64
    rows = []
    for r0 in range(0, A, G):
        r1 = min(A, r0 + G)
        rows += list(np.linspace(r0, r1 - 1, 64).round().astype(int))
    rows = np.array(sorted(set(rows + list(range(A - 64, A)))), np.int32)
    assert len(rows) >= 64 * st["groups"]
    idx = torch.as_tensor(rows.astype(np.int64), device=dev)
    _oracle_rows_check(g, rows, lat[idx].cpu().numpy(), rel[idx].cpu().numpy(),
                       hops[idx].cpu().numpy().astype(np.uint32), kind[idx].cpu().numpy())
