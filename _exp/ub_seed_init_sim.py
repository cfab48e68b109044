"""Sparse pull rounds SEEDED with hub upper bounds (r06 model; r04's ub_seed_sim.py used the
bounds only as an acceptance filter).  Jacobi rounds over one 64-source batch, as in
ub_seed_sim.py:

  plain : D = inf, D(s, s) = 0, the sources' out-neighbours active
  seeded: D(v, s) = (1 + 1e-9) * min_h (d(s, h) + d(h, v)) over the H top-degree hubs
          (an upper bound strictly above the true distance, so every reached pair still
          changes at least once, to a value from a real in-arc), D(s, s) = 0, and only the
          sources' out-neighbours active: a seed is not a change and activates nothing

A visit of (v, batch) reads every in-arc's tail row (64 lanes x 8 B = 512 B); the figure that
decides the sparse rounds' time is the row reads per (vertex, batch) (C4 measured 8.4 visits).
Also reported: reads of the 64-byte segments (8 lanes) that hold a lane whose tail changed
(what a per-segment change mask could skip), and the seeding's own cost (one hub batch, then a
min-plus product H deep per (vertex, source)).
usage: python3 _exp/ub_seed_init_sim.py [C4|C5] [hubs] [batches]"""
import sys
import numpy as np

sys.path.insert(0, '.')
from shadow_amd import synth

CFG = sys.argv[1] if len(sys.argv) > 1 else "C4"
NH = int(sys.argv[2]) if len(sys.argv) > 2 else 64
NB = int(sys.argv[3]) if len(sys.argv) > 3 else 2
g = synth.barabasi_albert() if CFG == "C4" else synth.chung_lu()
V = g.n
s, d, w = np.asarray(g.src), np.asarray(g.dst), np.asarray(g.latency)
keep = s != d
s, d, w = s[keep], d[keep], w[keep]
s, d = np.concatenate([s, d]), np.concatenate([d, s])
w = np.concatenate([w, w])
o = np.argsort(d, kind='stable')
s, d, w = s[o], d[o], w[o]
starts = np.searchsorted(d, np.arange(V))
indeg = np.diff(np.append(starts, len(d)))
has = indeg > 0
outdeg = np.bincount(s, minlength=V)


def rounds(srcs, D0=None):
    L = len(srcs)
    D = np.full((V, L), np.inf) if D0 is None else D0.copy()
    D[srcs, np.arange(L)] = 0.0
    changed = np.zeros((V, L), bool)
    changed[srcs, np.arange(L)] = True
    rows = segs = visits = 0.0
    pushes = 0.0  # push form: rows of the out-neighbours read for every (vertex, batch) that changed
    nr = 0
    for r in range(400):
        anych = changed.any(1)
        pushes += outdeg[anych].sum()
        act = np.zeros(V, bool)
        act[d[anych[s]]] = True
        visits += act.sum()
        rows += indeg[act].sum()
        # 64-byte segments of the tail rows that hold a changed lane, over the active visits
        segch = changed.reshape(V, L // 8, 8).any(2)          # [V, 8]
        arc_act = act[d]
        segs += segch[s[arc_act]].sum()
        c = D[s] + w[:, None]
        m = np.full((V, L), np.inf)
        m[has] = np.minimum.reduceat(c, starts[has], axis=0)
        m[~act] = np.inf                                       # only active vertices are visited
        newD = np.minimum(D, m)
        changed = newD < D
        D = newD
        nr += 1
        if not changed.any():
            break
    return D, nr, visits / V, rows / V, segs / V, pushes / V


rng = np.random.default_rng(1)
att = np.asarray(g.attached)
H = np.argsort(-outdeg)[:NH]
Dh, nrh, vh, rh, _, _ = rounds(H)                                # hub distances [V, NH] (one batch)
print(f"{CFG}: V={V} arcs={len(s)} hubs={NH}; hub batch {nrh} rounds, {rh:.2f} row reads per vertex")
tot = {"plain": np.zeros(5), "seeded": np.zeros(5)}
for bi in range(NB):
    srcs = np.sort(rng.choice(att, 64, replace=False))
    Dex, nr0, v0, r0, s0, p0 = rounds(srcs)
    UB = np.min(Dh[srcs][:, None, :] + Dh[None, :, :], axis=2).T * (1 + 1e-9)   # [V, 64]
    fin = np.isfinite(Dex) & (Dex > 0)
    tight = np.mean(UB[fin] <= Dex[fin] * 1.001), np.mean(UB[fin] <= Dex[fin] * 1.01)
    D1, nr1, v1, r1, s1, p1 = rounds(srcs, D0=UB)
    assert np.array_equal(D1, Dex), "seeded rounds reach another fixed point"
    print(f" batch {bi}: UB within 0.1% {tight[0]:.3f}, 1% {tight[1]:.3f}; rounds {nr0} -> {nr1}; "
          f"visits/vertex {v0:.2f} -> {v1:.2f}; row reads/vertex {r0:.2f} -> {r1:.2f}; "
          f"changed-segment reads/vertex {s0:.2f} -> {s1:.2f} (of 8 per row); push row reads/vertex {p0:.2f} -> {p1:.2f}")
    tot["plain"] += (nr0, v0, r0, s0, p0)
    tot["seeded"] += (nr1, v1, r1, s1, p1)
p, q = tot["plain"] / NB, tot["seeded"] / NB
print(f"mean: rounds {p[0]:.1f} -> {q[0]:.1f}; visits {p[1]:.2f} -> {q[1]:.2f}; row reads {p[2]:.2f} -> {q[2]:.2f} "
      f"({100 * (1 - q[2] / p[2]):.1f} % fewer); segment reads {p[3]:.2f} -> {q[3]:.2f} ({100 * (1 - q[3] / p[3]):.1f} % fewer); "
      f"push row reads {p[4]:.2f} -> {q[4]:.2f} (one pull pass: {len(s) / V:.2f})")
print(f"seeding cost: one hub batch ({rh:.2f} row reads per vertex, once per attached set) + a min-plus "
      f"product of depth {NH} per (vertex, source): {NH} f64 add+min per pair")
