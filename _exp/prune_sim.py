"""Ideal skip rate of the pruned dense sweep on C2 (thresholds = direct-arc latencies)."""
import numpy as np, sys
sys.path.insert(0, '.')
from shadow_amd import synth
V = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
A = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
mode = sys.argv[3] if len(sys.argv) > 3 else "landmark"
g = synth.geometric_complete_ish(V=V, A=A)
W = np.full((V, V), np.inf, np.float32)
W[g.src, g.dst] = g.latency; W[g.dst, g.src] = g.latency
np.fill_diagonal(W, np.inf)
def morton(cols):
    q = []
    for c in cols:
        c = np.where(np.isfinite(c), c, np.nanmax(np.where(np.isfinite(c), c, np.nan)))
        q.append(((c - c.min()) / (c.max() - c.min()) * (2**21 - 1)).astype(np.uint64))
    key = np.zeros(len(cols[0]), np.uint64)
    for b in range(21):
        for k, qq in enumerate(q):
            key |= ((qq >> np.uint64(b)) & np.uint64(1)) << np.uint64(b * len(q) + k)
    return key
def hilbert(x, y, order=16):
    n = 1 << order
    x = ((x - x.min()) / (x.max() - x.min()) * (n - 1)).astype(np.int64)
    y = ((y - y.min()) / (y.max() - y.min()) * (n - 1)).astype(np.int64)
    d = np.zeros(len(x), np.int64)
    sh = n // 2
    while sh > 0:
        rx = (x & sh) > 0; ry = (y & sh) > 0
        d += sh * sh * ((3 * rx) ^ ry)
        # rotate
        m = ~ry
        fl = m & rx
        x = np.where(fl, sh - 1 - x, x); y = np.where(fl, sh - 1 - y, y)
        x, y = np.where(m, y, x), np.where(m, x, y)
        sh //= 2
    return d.astype(np.uint64)
HIL = mode.endswith("h")
if HIL: mode = mode[:-1]
_morton = morton
def morton(cols):
    if HIL and len(cols) == 2: return hilbert(np.asarray(cols[0], np.float64), np.asarray(cols[1], np.float64))
    return _morton(cols)
if mode == "landmark":
    lm = [0]; 
    for _ in range(2):
        m = np.min(np.stack([np.where(np.isfinite(W[l]), W[l], 0) for l in lm]), 0); lm.append(int(np.argmax(m)))
    vkey = morton([W[l].astype(np.float64) for l in lm])
elif mode.startswith("pca"):
    nl = int(__import__("os").environ.get("NL", 8)); nc = int(mode[3:] or 2)
    lm = [0]
    while len(lm) < nl:
        m = np.min(np.stack([np.where(np.isfinite(W[l]), W[l], 0) for l in lm]), 0); m[lm] = -1; lm.append(int(np.argmax(m)))
    X = np.stack([np.where(np.isfinite(W[l]), W[l], np.nan).astype(np.float64) for l in lm], 1)
    X = np.where(np.isnan(X), np.nanmean(X, 0), X)
    X -= X.mean(0)
    ev, evec = np.linalg.eigh(X.T @ X)
    Y = X @ evec[:, ::-1][:, :nc]
    vkey = morton([Y[:, i] for i in range(nc)])
elif mode == "lmds":
    nl = 8
    lm = [0]
    while len(lm) < nl:
        m = np.min(np.stack([np.where(np.isfinite(W[l]), W[l], 0) for l in lm]), 0); m[lm] = -1; lm.append(int(np.argmax(m)))
    X = np.stack([np.where(np.isfinite(W[l]), W[l], np.nan).astype(np.float64) for l in lm], 1)
    X = np.where(np.isnan(X), np.nanmean(X, 0), X) ** 2
    Dl = X[lm]  # landmark x landmark squared distances
    Dl = (Dl + Dl.T) / 2
    H = np.eye(nl) - 1.0 / nl
    Bm = -0.5 * H @ Dl @ H
    ev, evec = np.linalg.eigh(Bm)
    Y = X @ evec[:, ::-1][:, :2]
    vkey = morton([Y[:, 0], Y[:, 1]])
else:
    r1 = np.random.default_rng(1); pts = r1.random((V, 2)); vkey = morton([pts[:, 0], pts[:, 1]])
perm = np.argsort(vkey, kind="stable")
att = g.attached
akey = vkey[att]; att = att[np.argsort(akey, kind="stable")]
Wp = W[np.ix_(perm, perm)]
nch = (V + 31) // 32; Vq = nch * 32
Wpp = np.full((Vq, Vq), np.inf, np.float32); Wpp[:V, :V] = Wp
minW = Wpp.reshape(nch, 32, Vq // 8, 8).min(axis=(1, 3))  # [chunk][wave tile]
tot = skip = 0
for b in range(0, len(att), 64):
    S = att[b:b + 64]
    Ds = np.full((len(S), Vq), np.inf, np.float32); Ds[:, :V] = W[np.ix_(S, perm)]
    for i, s in enumerate(S): Ds[i, np.where(perm == s)[0][0]] = np.inf
    minD = Ds.reshape(len(S), nch, 32).min(axis=2)  # [lane][chunk]
    Ts = Ds.copy()
    for i, s in enumerate(S):  # dropped pairs: two-hop distance (the sweep's tightened threshold)
        miss = np.where(~np.isfinite(Ts[i, :V]))[0]
        miss = miss[perm[miss] != s]
        if len(miss): Ts[i, miss] = (Ds[i, :V, None] + Wp[:, miss]).min(axis=0)
        Ts[i, np.where(perm == s)[0][0]] = 0
    tm = Ts.reshape(len(S), Vq // 8, 8).max(axis=2)  # [lane][wave tile], inf if any dropped
    # skip[c][w] iff all lanes: minD[l][c] + minW[c][w] > tm[l][w]
    ok = np.ones((nch, Vq // 8), bool)
    for l in range(len(S)):
        ok &= (minD[l][:, None] + minW) > tm[l][None, :]
    tot += ok.size; skip += ok.sum()
print(f"{mode}: ideal skip fraction {skip / tot:.3f} (tm incl. inf for dropped pairs)")
