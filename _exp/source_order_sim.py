"""Re-export C4.bin with the attached sources in another batch order (by distance to the
top hub, nearest of 8 hubs, random, degree, summed hub distances) for sched_sim_gs."""
import numpy as np, sys, struct, scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra
f = open('C4.bin','rb')
V = struct.unpack('i', f.read(4))[0]; M = struct.unpack('q', f.read(8))[0]
ptr = np.frombuffer(f.read(8*(V+1)), np.int64); src = np.frombuffer(f.read(4*M), np.int32); w = np.frombuffer(f.read(8*M), np.float64)
n = struct.unpack('i', f.read(4))[0]; att = np.frombuffer(f.read(4*n), np.int32)
dst = np.repeat(np.arange(V), np.diff(ptr))
G = sp.csr_matrix((w, (src, dst)), shape=(V, V))
deg = np.diff(ptr)
hubs = np.argsort(-deg)[:8]
D = dijkstra(G, indices=hubs)  # 8 x V
mode = sys.argv[1]
if mode == 'hub0':
    key = D[0, att]
elif mode == 'nearest':
    key = D[:, att].argmin(0) * 1e6 + D[:, att].min(0)
elif mode == 'random':
    key = np.random.default_rng(0).random(len(att))
elif mode == 'deg':
    key = -deg[att]
elif mode == 'sum':
    key = D[:, att].sum(0)
order = att[np.argsort(key, kind='stable')]
with open(f'C4_{mode}.bin', 'wb') as g:
    np.array([V], np.int32).tofile(g); np.array([M], np.int64).tofile(g)
    ptr.tofile(g); src.tofile(g); w.tofile(g)
    np.array([len(order)], np.int32).tofile(g); order.astype(np.int32).tofile(g)
