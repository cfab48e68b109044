#!/usr/bin/env python3
"""Offline model: would an f32-filtered sparse pull cut the row traffic of the lean rounds?

Jacobi Bellman-Ford rounds for one 64-source batch of a synthetic config.  Per round, for
every active destination v and in-arc (u, v) (a 512-byte row of d(u) over 64 lanes today),
count the lanes whose candidate d(u) + w could beat or tie v's current distance (they would
need the exact f64 row entry after an f32 filter), and the 64-byte / 128-byte segments of
the f64 row holding at least one such lane.  'pred' counts the lane whose stored predecessor
is u as passing (it ties unless d(u) fell); 'nopred' drops it when d(u) did not change in
the previous round (an exact per-lane change bit, a lower bound for stamp-based variants).
usage: _exp/sparse_f32_filter_sim.py [C4|C5|C3] [batch seed]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from shadow_amd import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
g = {"C4": lambda: synth.barabasi_albert(V=100_000, A=10_000), "C3": lambda: synth.knn_geographic(V=7_000),
     "C5": lambda: synth.chung_lu(V=1_000_000, A=50_000)}[cfg]()
V = g.n
keep = g.src != g.dst
s, d, w = g.src[keep], g.dst[keep], g.latency[keep]
if not g.directed:
    s, d, w = np.concatenate([s, d]), np.concatenate([d, s]), np.concatenate([w, w])
order = np.argsort(d, kind="stable")
tail, head, wt = s[order].astype(np.int64), d[order].astype(np.int64), w[order]
rng = np.random.default_rng(seed)
srcs = rng.choice(g.attached, 64, replace=False)
L = 64
D = np.full((V, L), np.inf)
D[srcs, np.arange(L)] = 0.0
pred = np.full((V, L), -1, np.int64)  # arc index
changed = np.zeros((V, L), bool)
changed[srcs, np.arange(L)] = True
tot = dict(rows=0, lanes=0, seg64_ch=0, rows_ch=0, lanes_ch=0, pass_pred=0, pass_nopred=0, seg64_pred=0, seg64_nopred=0, seg128_nopred=0, rows_any=0)
rnd = 0
E = len(tail)
CH = 1 << 18
while changed.any():
    # active destinations: any in-arc whose tail changed in the previous round (the GPU's
    # activation marks every out-neighbour of a changed vertex)
    act_v = np.zeros(V, bool)
    chv = changed.any(1)
    act_v[head[chv[tail]]] = True
    newD = D.copy()
    newP = pred.copy()
    r = dict(rows=0, seg64_ch=0, rows_ch=0, lanes_ch=0, pass_pred=0, pass_nopred=0, seg64_pred=0, seg64_nopred=0, seg128_nopred=0, rows_any=0)
    arcs = np.nonzero(act_v[head])[0]
    for a0 in range(0, len(arcs), CH):
        ai = arcs[a0:a0 + CH]
        u, v, ww = tail[ai], head[ai], wt[ai]
        c = D[u] + ww[:, None]
        cur = D[v]
        ok = c <= cur
        ok &= np.isfinite(c)
        ispred = pred[v] == ai[:, None]
        p_nopred = ok & ~(ispred & ~changed[u])
        r["rows"] += len(ai)
        r["pass_pred"] += int(ok.sum())
        r["pass_nopred"] += int(p_nopred.sum())
        r["seg64_pred"] += int(ok.reshape(len(ai), 8, 8).any(2).sum())
        r["seg64_nopred"] += int(p_nopred.reshape(len(ai), 8, 8).any(2).sum())
        r["seg128_nopred"] += int(p_nopred.reshape(len(ai), 4, 16).any(2).sum())
        r["rows_any"] += int(p_nopred.any(1).sum())
        chu = changed[u]  # lanes whose tail value changed last round (a per-lane change mask)
        r["lanes_ch"] += int(chu.sum())
        r["seg64_ch"] += int(chu.reshape(len(ai), 8, 8).any(2).sum())
        r["rows_ch"] += int(chu.any(1).sum())
        # Jacobi update (min over arcs): process strictly better candidates
        better = c < newD[v]
        if better.any():
            ii, ll = np.nonzero(better)
            # several arcs of one chunk may hit the same (v, lane): take the minimum
            key = v[ii] * L + ll
            o = np.lexsort((c[ii, ll], key))
            key, ii, ll = key[o], ii[o], ll[o]
            first = np.ones(len(key), bool)
            first[1:] = key[1:] != key[:-1]
            ii, ll = ii[first], ll[first]
            vv = v[ii]
            m = c[ii, ll] < newD[vv, ll]
            newD[vv[m], ll[m]] = c[ii, ll][m]
            newP[vv[m], ll[m]] = ai[ii][m]
    changed = newD < D
    D, pred = newD, newP
    for k in r:
        tot[k] += r[k]
    nr = max(r["rows"], 1)
    print(f"round {rnd:2d} rows {r['rows']:9d} lanes/row pass {r['pass_pred'] / nr:5.2f} (no pred {r['pass_nopred'] / nr:5.2f})"
          f"  64B segs/row {r['seg64_pred'] / nr:4.2f} ({r['seg64_nopred'] / nr:4.2f})  128B {r['seg128_nopred'] / nr:4.2f}"
          f"  rows w/ any {r['rows_any'] / nr:4.2f}  changed lanes/row {r['lanes_ch'] / nr:5.2f} segs {r['seg64_ch'] / nr:4.2f}"
          f" rows {r['rows_ch'] / nr:4.2f}", flush=True)
    rnd += 1
nr = tot["rows"]
print(f"total rows {nr}  lanes/row {tot['pass_pred'] / nr:.2f} (no pred {tot['pass_nopred'] / nr:.2f})  "
      f"64B segs/row {tot['seg64_pred'] / nr:.2f} of 8 ({tot['seg64_nopred'] / nr:.2f})  128B {tot['seg128_nopred'] / nr:.2f} of 4")
# bytes per row visit: today 512; filtered: 256 (f32 row) + 64 x segs
print(f"changed lanes/row {tot['lanes_ch'] / nr:.2f}  64B segs/row {tot['seg64_ch'] / nr:.2f}  rows {tot['rows_ch'] / nr:.2f}")
print(f"bytes/row per-lane change masks: {64 * tot['seg64_ch'] / nr + 8:.0f} (segments + one 8-byte mask)")
for lab, sg in (("pred", tot["seg64_pred"]), ("nopred", tot["seg64_nopred"])):
    print(f"bytes/row today 512  f32 filter ({lab}) {256 + 64 * sg / nr:.0f}")
