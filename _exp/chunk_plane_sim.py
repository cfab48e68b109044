"""Pruned C2 sweep, offline model (r06): a chunk bound from supporting planes instead of the
box.  For a 32-row chunk C, a lane (source s) and a column (destination t):

  box   : min_u D(s,u) + W(u,t)  >=  min_u D(s,u) + min_u W(u,t)                (the kernel's)
  plane : D(s,u) >= p_s + a_s . x_u,  W(u,t) >= q_t + b_t . x_u   for every u in C
          (p_s = min_u D(s,u) - a_s . x_u, q_t likewise: valid for ANY slopes a_s, b_t), so
          min_u D + W >= p_s + q_t + min_{x in box(C)} (a_s + b_t) . x
          (x_u: a per-row feature, here 2 coordinates; the box of the chunk's rows in them)

Exact for any graph (a bad embedding only makes it loose; a = b = 0 is the box bound).  The
slopes are least-squares fits over the chunk's rows.  Reports the fraction of chunks each
bound leaves live for a block (32 destinations x 64 sources) under the FINAL thresholds (the
floor of the sweep's work), next to the exact fraction.
usage: python3 _exp/chunk_plane_sim.py [V] [coords: true|mds|land] [landmarks] [trials]
(land: the features are the NL landmark distances, the chunk order the landmark-MDS Hilbert one)"""
import sys
import numpy as np
from scipy.sparse.csgraph import dijkstra

V = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
COORDS = sys.argv[2] if len(sys.argv) > 2 else "true"
NL = int(sys.argv[3]) if len(sys.argv) > 3 else 3
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
Wz = np.where(np.isinf(W), 0, W)

if COORDS == "true":
    X = pts.copy()
    L = None
else:
    # landmark MDS as the engine's locality order does: farthest-point landmarks, their
    # distance vectors centred, the top two principal axes
    land = [0]
    dl = [dijkstra(Wz, indices=0)]
    mind = dl[0].copy()
    for _ in range(NL - 1):
        nxt = int(np.argmax(np.where(np.isfinite(mind), mind, -1)))
        land.append(nxt)
        dl.append(dijkstra(Wz, indices=nxt))
        mind = np.minimum(mind, dl[-1])
    L = np.stack(dl, 1)
    Lc = L - L.mean(0)
    _, _, vt = np.linalg.svd(Lc, full_matrices=False)
    X = Lc @ vt[:2].T
X = (X - X.min(0)) / (X.max(0) - X.min(0))
ORDER = X
if COORDS == "land":
    # the plane features are the landmark distances themselves (NL dims), the order the MDS one
    X = (L - L.min(0)) / (L.max(0) - L.min(0))


def hilbert(x, y, n=1 << 10):
    x = (x * (n - 1)).astype(np.int64)
    y = (y * (n - 1)).astype(np.int64)
    dd = np.zeros_like(x)
    s = n >> 1
    while s > 0:
        rx = ((x & s) > 0).astype(np.int64)
        ry = ((y & s) > 0).astype(np.int64)
        dd += s * s * ((3 * rx) ^ ry)
        m = ry == 0
        f = m & (rx == 1)
        x = np.where(f, n - 1 - x, x)
        y = np.where(f, n - 1 - y, y)
        x2 = np.where(m, y, x)
        y = np.where(m, x, y)
        x = x2
        s >>= 1
    return dd


perm = np.argsort(hilbert(ORDER[:, 0], ORDER[:, 1]), kind="stable")
rng = np.random.default_rng(5)
SRS, BW = 32, 32
nch = V // SRS


def fit_planes(M, Xc):
    """rows of M (n_lanes x 32 rows): least-squares slopes over the finite entries, then the
    supporting offset p = min_u (M - a.x_u); returns p, a (n x 2)"""
    n = M.shape[0]
    a = np.zeros((n, Xc.shape[1]))
    fin = np.isfinite(M)
    A1 = np.concatenate([Xc, np.ones((Xc.shape[0], 1))], 1)
    for i in range(n):
        f = fin[i]
        if f.sum() >= Xc.shape[1] + 2:
            sol, *_ = np.linalg.lstsq(A1[f], M[i, f], rcond=None)
            a[i] = sol[:-1]
    p = np.min(np.where(fin, M - a @ Xc.T, np.inf), axis=1)
    return p, a


res = {"box": [], "plane": [], "plane|box": [], "exact": []}
for trial in range(int(sys.argv[4]) if len(sys.argv) > 4 else 4):
    c = pts[rng.integers(V)]
    S = np.argsort(((pts - c) ** 2).sum(1))[:64]
    Dfin = dijkstra(Wz, indices=S)
    D0 = W[S]
    tiles = rng.integers(0, V // BW, 6)
    for tt in tiles:
        tv = perm[tt * BW:(tt + 1) * BW]
        T = Dfin[:, tv]
        live = {k: 0 for k in res}
        for ch in range(nch):
            rows = perm[ch * SRS:(ch + 1) * SRS]
            Xr = X[rows]
            ctr = 0.5 * (Xr.min(0) + Xr.max(0))
            h = 0.5 * (Xr.max(0) - Xr.min(0))
            Xc = Xr - ctr
            Dm = D0[:, rows]                     # [64, 32]
            Wm = W[np.ix_(rows, tv)].T           # [32 dests, 32 rows]
            md = Dm.min(1)
            mw = Wm.min(1)
            box = md[:, None] + mw[None, :]
            p, a = fit_planes(Dm, Xc)
            q, b = fit_planes(Wm, Xc)
            g = a[:, None, :] + b[None, :, :]    # [64, 32, 2]
            plane = p[:, None] + q[None, :] - (np.abs(g) * h).sum(2)
            cand = Dm[:, :, None] + W[np.ix_(rows, tv)][None, :, :]
            exact = cand.min(1)
            live["box"] += bool((box <= T).any())
            live["plane"] += bool((plane <= T).any())
            live["plane|box"] += bool(((np.maximum(plane, box)) <= T).any())
            live["exact"] += bool((exact <= T).any())
            assert (np.maximum(plane, box)[np.isfinite(exact)] <= exact[np.isfinite(exact)] + 1e-9).all()
        for k in res:
            res[k].append(live[k] / nch)
print(f"V={V} coords={COORDS} NL={NL}")
for k, v in res.items():
    print(f"{k:10s} live chunk fraction mean {np.mean(v):.3f} (min {np.min(v):.3f}, max {np.max(v):.3f})")
