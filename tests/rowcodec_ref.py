"""A CPU row codec with the engine's payload format (shadowtopo_pack_rows, engine.hip), for the
gloo tests of shard.RowExchange's packed exchange (the engine's codec needs a GPU; its own
round trip is checked in tests/test_engine_gpu.py).  Test infrastructure only.

Payload: header {u64 explicit pairs, u64 words} | mask[words] u64 | prefix[words] u32,
padded to 16 bytes | explicit entries {f64 lat, f64 rel, u32 hops, u32 0} in pair order.
A set mask bit means the pair equals recon(s, t), which every rank computes from its own
copy of the graph (here: the lightest arc s -> t, latency 0 + w, one hop, reliability
vfac(s) * (1 - loss)); whatever recon returns, a pair that differs is sent in full."""
from __future__ import annotations

import numpy as np
import torch


def _words(pairs):
    return (pairs + 63) // 64


def _entry_off(w):
    return (16 + w * 8 + w * 4 + 15) // 16 * 16


class RefRowCodec:
    def __init__(self, g):
        n = g.n
        self.W = np.full((n, n), np.inf)
        self.WR = np.zeros((n, n))
        for s, t, w, p in zip(g.src, g.dst, g.latency, g.packetloss):
            for a, b in ((s, t), (t, s)) if not g.directed else ((s, t),):
                if w < self.W[a, b]:
                    self.W[a, b] = w
                    self.WR[a, b] = 1.0 - p
        vl = g.vertex_packetloss
        self.vfac = np.ones(n) if vl is None else np.where(np.isnan(vl), 1.0, 1.0 - np.nan_to_num(vl))
        self.att = np.asarray(g.attached, np.int64)

    def capacity(self, rows, A):
        pairs = rows * A
        return (_entry_off(_words(pairs)) + pairs * 24 + 255) // 256 * 256

    def _recon(self, a, z):
        s = self.att[a:z][:, None]
        t = self.att[None, :]
        w = self.W[s, t]
        ok = np.isfinite(w) & (s != t)
        lat = np.where(ok, 0.0 + w, 0.0)
        rel = np.where(ok, self.vfac[s] * self.WR[s, t], 0.0)
        return ok.ravel(), lat.ravel(), rel.ravel()

    def pack(self, a, z, lat, rel, hops, out) -> int:
        pairs = (z - a) * len(self.att)
        nw = _words(pairs)
        ok, rl, rr = self._recon(a, z)
        L = lat.reshape(-1).numpy()[:pairs]
        R = rel.reshape(-1).numpy()[:pairs]
        H = hops.reshape(-1).numpy().view(np.uint32)[:pairs]
        same = ok & (H == 1) & (L.view(np.uint64) == rl.view(np.uint64)) & (R.view(np.uint64) == rr.view(np.uint64))
        bits = np.zeros(nw * 64, bool)
        bits[:pairs] = same
        mask = np.bitwise_or.reduce(bits.reshape(nw, 64).astype(np.uint64) << np.arange(64, dtype=np.uint64), axis=1)
        expl = np.nonzero(~same)[0]
        cnt = np.zeros(nw * 64, np.int64)
        cnt[:pairs] = ~same
        prefix = np.concatenate([[0], np.cumsum(cnt.reshape(nw, 64).sum(1))[:-1]]).astype(np.uint32)
        buf = out.numpy()
        buf[:16] = np.frombuffer(np.array([len(expl), nw], np.uint64).tobytes(), np.uint8)
        buf[16:16 + nw * 8] = np.frombuffer(mask.tobytes(), np.uint8)
        buf[16 + nw * 8:16 + nw * 12] = np.frombuffer(prefix.tobytes(), np.uint8)
        e = np.zeros(len(expl), dtype=[("lat", "<f8"), ("rel", "<f8"), ("hops", "<u4"), ("pad", "<u4")])
        e["lat"], e["rel"], e["hops"] = L[expl], R[expl], H[expl]
        o = _entry_off(nw)
        buf[o:o + e.nbytes] = np.frombuffer(e.tobytes(), np.uint8)
        return (o + e.nbytes + 255) // 256 * 256

    def unpack(self, a, z, payload, lat, rel, hops):
        pairs = (z - a) * len(self.att)
        nw = _words(pairs)
        buf = payload.numpy()
        mask = np.frombuffer(buf[16:16 + nw * 8].tobytes(), np.uint64)
        bits = ((mask[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool).ravel()[:pairs]
        prefix = np.frombuffer(buf[16 + nw * 8:16 + nw * 12].tobytes(), np.uint32).astype(np.int64)
        o = _entry_off(nw)
        n_expl = int(np.frombuffer(buf[:8].tobytes(), np.uint64)[0])
        e = np.frombuffer(buf[o:o + 24 * n_expl].tobytes(),
                          dtype=[("lat", "<f8"), ("rel", "<f8"), ("hops", "<u4"), ("pad", "<u4")])
        idx = np.nonzero(~bits)[0]
        # the k-th explicit pair of word w is entry prefix[w] + k
        rank_in_word = np.cumsum(~bits) - 1
        base = prefix[np.arange(pairs) // 64]
        first = np.zeros(pairs, np.int64)
        starts = np.arange(0, pairs, 64)
        before = np.concatenate([[0], np.cumsum(~bits)])[starts]
        first[:] = np.repeat(before, 64)[:pairs]
        k = base + rank_in_word - first
        ok, rl, rr = self._recon(a, z)
        L = rl.copy()
        R = rr.copy()
        H = np.ones(pairs, np.uint32)
        L[idx] = e["lat"][k[idx]]
        R[idx] = e["rel"][k[idx]]
        H[idx] = e["hops"][k[idx]]
        lat.reshape(-1)[:pairs] = torch.from_numpy(L)
        rel.reshape(-1)[:pairs] = torch.from_numpy(R)
        hops.reshape(-1)[:pairs] = torch.from_numpy(H.view(np.int32))


class RefHopCodec:
    """CPU stand-in of shard.EngineHopCodec (shadowtopo_hops_narrow / _widen): u32 hop counts
    -> low / high 16-bit halves, overflow word OR-ed with 1 when a count is >= 2^16"""

    def narrow(self, hops, lo, hi, overflow):
        h = hops.reshape(-1).numpy().view(np.uint32)
        lo.reshape(-1).numpy().view(np.uint16)[:] = (h & 0xFFFF).astype(np.uint16)
        if hi is not None:
            hi.reshape(-1).numpy().view(np.uint16)[:] = (h >> 16).astype(np.uint16)
        if (h >> 16).any():
            overflow[0] |= 1

    def widen(self, lo, hi, out):
        v = lo.reshape(-1).numpy().view(np.uint16).astype(np.uint32)
        if hi is not None:
            v |= hi.reshape(-1).numpy().view(np.uint16).astype(np.uint32) << 16
        out.reshape(-1).numpy().view(np.uint32)[:] = v
