"""Pruned C2 sweep: which 32-row chunks a block (32 destinations x 64 sources) must visit
under its FINAL thresholds (a lower bound on the sweep's work), with every pair and with the
pairs that have no direct arc left out -- does one kind of pair hold the chunks live?"""
import sys
import numpy as np
from scipy.sparse.csgraph import dijkstra
sys.path.insert(0, '/root/repo')
V = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
r1 = np.random.default_rng(1)
pts = r1.random((V, 2))
r2 = np.random.default_rng(2)
d = np.sqrt(((pts[:, None, :] - pts[None, :, :]) ** 2).sum(2))
W = 1.0 + 200.0 * d + r1.uniform(0, 1e-3, (V, V))
W = np.minimum(W, W.T)
drop = r2.random((V, V)) < 0.05
drop = np.triu(drop, 1)
drop = drop | drop.T
W[drop] = np.inf
np.fill_diagonal(W, np.inf)
# Hilbert-ish order: sort by a Morton key of the coordinates
q = (pts * 1024).astype(np.int64)
def morton(x, y):
    k = np.zeros_like(x)
    for b in range(10):
        k |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
    return k
perm = np.argsort(morton(q[:, 0], q[:, 1]), kind='stable')
rng = np.random.default_rng(5)
SRS, BW = 32, 32
nch = V // SRS
res = {"all": [], "arc_only": [], "sub2": [], "sub4": [], "sub8": [], "exact": []}
for trial in range(6):
    c = pts[rng.integers(V)]
    S = np.argsort(((pts - c) ** 2).sum(1))[:64]            # a locality batch
    Dfin = dijkstra(np.where(np.isinf(W), 0, W), indices=S)   # [64, V] exact (0 = no edge in csgraph)
    D0 = W[S]                                                  # seeds: direct arcs
    tiles = rng.integers(0, V // BW, 8)
    for tt in tiles:
        tv = perm[tt * BW:(tt + 1) * BW]                       # the block's destinations
        T = Dfin[:, tv]                                        # [64, 32]
        arc = np.isfinite(W[np.ix_(S, tv)])
        for name, mask in (("all", np.ones_like(arc)), ("arc_only", arc)):
            live = 0
            for ch in range(nch):
                rows = perm[ch * SRS:(ch + 1) * SRS]
                md = np.min(D0[:, rows], axis=1)               # [64]
                mw = np.min(W[np.ix_(rows, tv)], axis=0)       # [32]
                ok = (md[:, None] + mw[None, :] <= T) & mask
                live += bool(ok.any())
            res[name].append(live / nch)
        live = 0
        for ch in range(nch):
            rows = perm[ch * SRS:(ch + 1) * SRS]
            c = D0[:, rows][:, :, None] + W[np.ix_(rows, tv)][None, :, :]   # [64, 32 rows, 32 dests]
            live += bool((c <= T[:, None, :]).any())
        res["exact"].append(live / nch)
        for ns in (2, 4, 8):
            live = 0
            for ch in range(nch):
                rows = perm[ch * SRS:(ch + 1) * SRS]
                ok = np.zeros_like(arc)
                for sg in np.split(rows, ns):
                    md = np.min(D0[:, sg], axis=1)
                    mw = np.min(W[np.ix_(sg, tv)], axis=0)
                    ok |= md[:, None] + mw[None, :] <= T
                live += bool(ok.any())
            res[f"sub{ns}"].append(live / nch)
for k, v in res.items():
    print(k, 'live chunk fraction mean %.3f (min %.3f, max %.3f)' % (np.mean(v), np.min(v), np.max(v)))
