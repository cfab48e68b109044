"""Export a config's relaxation in-CSR (loops dropped, parallel arcs merged to their minimum)
and attached list for the offline schedule models: python export_csr.py C4 [scale] -> C4.bin"""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
from shadow_amd import synth
cfg = sys.argv[1]; scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
g = synth.CONFIGS[cfg](scale)
V = g.n
s, d, w = g.src, g.dst, g.latency
nl = s != d
s, d, w = s[nl], d[nl], w[nl]
# undirected: arcs both ways; merge parallel by min
a = np.concatenate([s, d]); b = np.concatenate([d, s]); ww = np.concatenate([w, w])
key = b.astype(np.int64) * V + a
o = np.lexsort((ww, key))
key, a, b, ww = key[o], a[o], b[o], ww[o]
first = np.ones(len(key), bool); first[1:] = key[1:] != key[:-1]
a, b, ww = a[first], b[first], ww[first]
ptr = np.zeros(V + 1, np.int64); np.add.at(ptr, b + 1, 1); ptr = np.cumsum(ptr)
att = g.attached.astype(np.int32)
with open(f'{cfg}.bin', 'wb') as f:
    np.array([V], np.int32).tofile(f); np.array([len(a)], np.int64).tofile(f)
    ptr.tofile(f); a.astype(np.int32).tofile(f); ww.astype(np.float64).tofile(f)
    np.array([len(att)], np.int32).tofile(f); att.tofile(f)
print(V, len(a), len(att))
