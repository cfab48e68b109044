"""Activity of pull rounds on C4 with and without hub upper-bound seeding (simulation)."""
import sys, numpy as np
sys.path.insert(0, '.')
from shadow_amd import synth
g = synth.barabasi_albert()
V = g.n
s, d, w = np.asarray(g.src), np.asarray(g.dst), np.asarray(g.latency)
keep = s != d
s, d, w = s[keep], d[keep], w[keep]
s, d = np.concatenate([s, d]), np.concatenate([d, s]); w = np.concatenate([w, w])
o = np.argsort(d, kind='stable'); s, d, w = s[o], d[o], w[o]
starts = np.searchsorted(d, np.arange(V)); has = np.diff(np.append(starts, len(d))) > 0
outdeg = np.bincount(s, minlength=V)

def rounds(srcs, D0=None, verbose=True, UBF=None):
    L = len(srcs)
    D = np.full((V, L), np.inf) if D0 is None else D0.copy()
    D[srcs, np.arange(L)] = 0.0
    changed = np.zeros((V, L), bool); changed[srcs, np.arange(L)] = True
    stats = []
    for r in range(60):
        act_item = np.zeros(V, bool)
        anych = changed.any(1)
        act_item[d[anych[s]]] = True  # destinations of changed tails
        # per-lane activity: lane's tail changed
        lane_act = np.zeros((V, L), bool)
        np.logical_or.at(lane_act, d[anych[s]], changed[s[anych[s]]])
        c = D[s] + w[:, None]
        m = np.full((V, L), np.inf)
        m[has] = np.minimum.reduceat(c, starts[has], axis=0)
        newD = np.minimum(D, m) if UBF is None else np.where((m < D) & (m <= UBF), m, D)
        changed = newD < D
        stats.append((r, act_item.mean(), lane_act.mean(), changed.mean()))
        D = newD
        if not changed.any(): break
    if verbose:
        for st in stats: print('  round %2d items %.3f lanes %.4f changed %.4f' % st)
    return D, stats

rng = np.random.default_rng(1)
srcs = np.sort(rng.choice(np.asarray(g.attached), 64, replace=False))
print('plain')
Dex, st0 = rounds(srcs)
H = np.argsort(-outdeg)[:int(sys.argv[1]) if len(sys.argv) > 1 else 64]
Dh, _ = rounds(H, verbose=False)  # [V, H]
UB = np.min(Dh[srcs][:, None, :] + Dh[None, :, :], axis=2).T * (1 + 1e-9)  # [V, L]
print('UB tightness: exact fraction within 1%%: %.3f, 10%%: %.3f' % (np.mean(UB <= Dex * 1.01), np.mean(UB <= Dex * 1.1)))
print('UB filter')
D1, st1 = rounds(srcs, None, UBF=UB)
assert np.allclose(D1, Dex)
print('sum items plain %.2f seeded %.2f ; lanes %.3f vs %.3f' % (sum(x[1] for x in st0), sum(x[1] for x in st1), sum(x[2] for x in st0), sum(x[2] for x in st1)))
