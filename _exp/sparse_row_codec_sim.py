"""Sparse row exchange (r06 model): how far below 20 B per pair could a lossless codec take C4's
rows?  Rows of the attached-pair matrix (lat f64, rel f64, hops u32) from the oracle for a
sample of sources, then per field:
  raw          : 8 / 8 / 4 bytes
  hops16       : hops as u16 (what shard.EngineHopCodec sends: 18 B per pair)
  xor-prev     : Gorilla-style XOR with the previous pair of the row, leading/trailing zero
                 counts + the meaningful bits (a per-value bit cost; a GPU form would need a
                 prefix sum over the bit lengths and a bit-level scatter)
  byte-shuffle+zlib : the 8 byte planes of the row compressed separately (an entropy proxy)
usage: python3 _exp/sparse_row_codec_sim.py [sources]"""
import sys
import zlib

import numpy as np

sys.path.insert(0, '.')
from oracle import oracle as O
from shadow_amd import synth

n_src = int(sys.argv[1]) if len(sys.argv) > 1 else 16
g = synth.barabasi_albert()
og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss)
lat, rel, hops, kind, _ = og.pair_rows(og.flags(), g.attached, 0, n_src, nthreads=8)
og.close()


def xor_bits(v):
    u = v.view(np.uint64)
    x = u[1:] ^ u[:-1]
    bits = np.zeros(len(x))
    nz = x != 0
    lz = np.array([64 - int(t).bit_length() for t in x[nz]])
    tz = np.array([(int(t) & -int(t)).bit_length() - 1 for t in x[nz]])
    bits[~nz] = 1
    bits[nz] = 2 + 5 + 6 + (64 - lz - tz)
    return (64 + bits.sum()) / len(u) / 8


def shuffle_zlib(v):
    b = v.view(np.uint8).reshape(-1, 8)
    return sum(len(zlib.compress(b[:, k].tobytes(), 6)) for k in range(8)) / len(v)


tot = {"raw": 0.0, "hops16": 0.0, "xor": 0.0, "zlib": 0.0}
for r in range(n_src):
    L, R, H = lat[r], rel[r], hops[r]
    tot["raw"] += 20
    tot["hops16"] += 18
    tot["xor"] += xor_bits(L) + xor_bits(R) + 2
    tot["zlib"] += shuffle_zlib(L) + shuffle_zlib(R) + len(zlib.compress(H.astype(np.uint16).tobytes(), 6)) / len(H)
print(f"C4, {n_src} source rows x {lat.shape[1]} targets: max hops {int(hops.max())}")
for k, v in tot.items():
    print(f"  {k:7s} {v / n_src:6.2f} B per pair")
