"""Second, independent restatement of the parity-unpinned branch (TEST INFRASTRUCTURE ONLY:
never imported by the product).

igraph is absent from this image, so the shortest-path branch of the
reference -- igraph_get_shortest_paths_dijkstra called at
/root/reference/src/main/routing/topology.c:1754-1775 and the path fold of
_topology_computePathProperties (topology.c:1407-1523) -- cannot be run here.  The C oracle
(oracle/topo_oracle.c) restates it; this module restates it a second time, in plain Python,
written from igraph's published algorithm as SURVEY.md 8.0 records it (igraph 0.7.1 / 0.8.0,
src/paths/dijkstra.c and src/core/indheap.c, the indexed two-way heap), not from the C code:

  * incidence order (igraph_incident): undirected -- every edge at v sorted by (other end,
    edge id), a self-loop listed twice; directed OUT -- out-edges sorted by (head, edge id);
  * dists start at -1 (unseen), parents hold the edge; the heap is a max-heap on -dist;
    shift_up moves an element up unless it is strictly below its parent (equal keys move
    up); sink takes the left child when left >= right and swaps only when the parent is
    strictly below the child; modify = set + sink + shift_up; pop = switch root and last,
    shrink, sink the root;
  * relaxation in incidence order: an unseen head gets its first distance and the parent
    edge and is pushed; a seen one is updated only on a strictly smaller distance;
  * early exit once every target (the attached vertices, the source included) was popped.

Pair values (topology.c:1407-1523, 1848-1852): the vertex path from the parents; latency =
left fold from 0.0 of the latencies of the get_eid edge (lowest id) of each hop, 0 -> 1;
reliability = ((1 * (1 - lv_s)) * (1 - lv_t)) * prod(1 - loss_e) in path order (vertex loss
only where the attribute is present); hops = |path| - 1.

Cross-checked against topo_oracle.c on the integer-tie fixtures in tests/test_oracle.py
(predecessor edges and the pair rows).  Pure-Python loops: small graphs only.
"""
from __future__ import annotations

import math


class TwoWayHeap:
    """igraph_2wheap: keys in data[], heap position -> vertex in idx[], vertex -> position in pos"""

    def __init__(self):
        self.data = []
        self.idx = []
        self.pos = {}

    def __len__(self):
        return len(self.data)

    def _switch(self, a, b):
        if a == b:
            return
        self.data[a], self.data[b] = self.data[b], self.data[a]
        va, vb = self.idx[a], self.idx[b]
        self.idx[a], self.idx[b] = vb, va
        self.pos[vb] = a
        self.pos[va] = b

    def _shift_up(self, e):
        while e != 0:
            p = (e + 1) // 2 - 1
            if self.data[e] < self.data[p]:
                return
            self._switch(e, p)
            e = p

    def _sink(self, h):
        n = len(self.data)
        while True:
            left, right = 2 * h + 1, 2 * h + 2
            if left >= n:
                return
            c = left if (right == n or self.data[left] >= self.data[right]) else right
            if self.data[h] < self.data[c]:
                self._switch(h, c)
                h = c
            else:
                return

    def push(self, v, key):
        self.data.append(key)
        self.idx.append(v)
        self.pos[v] = len(self.data) - 1
        self._shift_up(len(self.data) - 1)

    def pop_max(self):
        v, key = self.idx[0], self.data[0]
        self._switch(0, len(self.data) - 1)
        self.data.pop()
        self.idx.pop()
        del self.pos[v]
        if self.data:
            self._sink(0)
        return v, key

    def modify(self, v, key):
        e = self.pos[v]
        self.data[e] = key
        self._sink(e)
        self._shift_up(e)


class RefGraph:
    def __init__(self, n, src, dst, latency, packetloss, vertex_packetloss=None, directed=False):
        self.n = int(n)
        self.src = [int(x) for x in src]
        self.dst = [int(x) for x in dst]
        self.lat = [float(x) for x in latency]
        self.loss = [float(x) for x in packetloss]
        self.vloss = None if vertex_packetloss is None else [float(x) for x in vertex_packetloss]
        self.directed = bool(directed)
        inc = [[] for _ in range(self.n)]
        for e, (a, b) in enumerate(zip(self.src, self.dst)):
            if self.directed:
                inc[a].append((b, e))
            elif a == b:
                inc[a].append((a, e))
                inc[a].append((a, e))  # a loop is incident twice
            else:
                inc[a].append((b, e))
                inc[b].append((a, e))
        self.inc = [sorted(x) for x in inc]
        self._eid = {}
        for e, (a, b) in enumerate(zip(self.src, self.dst)):
            k = (a, b) if self.directed else (min(a, b), max(a, b))
            self._eid.setdefault(k, e)  # lowest id first

    def get_eid(self, a, b):
        k = (a, b) if self.directed else (min(a, b), max(a, b))
        return self._eid.get(k, -1)

    def other(self, e, v):
        a, b = self.src[e], self.dst[e]
        return b if a == v else a

    def dijkstra(self, s, targets):
        """(dist, parent edge) with dist -1 where unseen; the heap history decides ties"""
        dist = [-1.0] * self.n
        parent = [-1] * self.n
        tgt = set(int(t) for t in targets)
        to_reach = len(tgt)
        dist[s] = 0.0
        h = TwoWayHeap()
        h.push(s, -0.0)
        while len(h) and to_reach > 0:
            u, key = h.pop_max()
            du = -key
            if u in tgt:
                tgt.discard(u)
                to_reach -= 1
            for (_, e) in self.inc[u]:
                x = self.other(e, u) if not self.directed else self.dst[e]
                alt = du + self.lat[e]
                cur = dist[x]
                if cur < 0:
                    dist[x] = alt
                    parent[x] = e
                    h.push(x, -alt)
                elif alt < cur:
                    dist[x] = alt
                    parent[x] = e
                    h.modify(x, -alt)
        return dist, parent

    def path(self, s, t, parent):
        p = [t]
        x = t
        while x != s:
            e = parent[x]
            if e < 0:
                return None
            x = self.other(e, x) if not self.directed else self.src[e]
            p.append(x)
        return p[::-1]

    def vfac(self, v):
        if self.vloss is None or math.isnan(self.vloss[v]):
            return None
        return 1.0 - self.vloss[v]

    def pair(self, s, t, parent):
        """shortest-path rule for s != t: (lat, rel, hops) or None when unreachable"""
        p = self.path(s, t, parent)
        if p is None:
            return None
        lat, rel = 0.0, 1.0
        fs, ft = self.vfac(s), self.vfac(t)
        if fs is not None:
            rel *= fs
        if ft is not None:
            rel *= ft
        for a, b in zip(p[:-1], p[1:]):
            e = self.get_eid(a, b)
            lat += self.lat[e]
            rel *= 1.0 - self.loss[e]
        if lat == 0:
            lat = 1.0
        return lat, rel, len(p) - 1
