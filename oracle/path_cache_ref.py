"""Test infrastructure (never imported by the product): a restatement of the reference's
path cache -- which attached pairs Shadow 1.14 has cached, in which direction, after a
sequence of queries -- so the tests can say what the drop-in getters must return.

It follows /root/reference/src/main/routing/topology.c:
  _topology_getPathEntry            :1969-2051  (cache lookup (s, t), then (t, s) when
                                                 undirected; on a miss: direct lookup,
                                                 self path or one Dijkstra from s; after a
                                                 successful one (s, t), then (t, s) in ANY
                                                 graph, :2033-2038)
  _topology_getPathFromCache        :1284-1303
  _topology_shouldStorePath         :1305-1334
  _topology_storePathInCache        :1336-1386  (running minimum -> worker_updateMinTimeJump)
  _topology_computeSourcePaths      :1655-1875  (stores every reachable attached target)
  _topology_computeShortestPathToSelf :1545-1653
  _topology_lookupDirectPath        :1877-1927

The path VALUES come from the caller (the oracle's own-row matrix: entry (s, t) is what
s's own computation gives), so this module decides only which entry a query sees.
Self pairs: igraph's path to the source itself is [] or [s] by version.  With
[] (the default rule) a Dijkstra run stores nothing for the source (topology.c:1815) and a
self pair is cached only by a query (s, s), through the self-path rule.  With [s]
(self_loop_rule) the run stores the source's self-loop path (the matrix diagonal), and fails
(after storing the rest) when the source has no self-loop; a query (s, s) that comes first
caches the self-path rule's value instead (self_lat / self_rel / self_kind).
"""
from __future__ import annotations

import numpy as np


class RefPathCache:
    def __init__(self, lat, kind, *, directed, complete, prefer_direct, adjacent, self_loop_rule=False,
                 self_lat=None, self_kind=None):
        """lat / kind: [A, A] oracle matrices over attached indices (kind 0 = unroutable);
        adjacent(i, j): the graph has an edge i -> j (either way when undirected; i == j:
        a self-loop).  In a directed graph too, _topology_shouldStorePath refuses (s, t) once
        (t, s) is cached (topology.c:1311-1317); the query (s, t) then misses every time
        (a directed lookup tries (s, t) only), reruns s's Dijkstra, and returns the (t, s)
        Path through the post-computation fallback (:2033-2038)."""
        self.lat = np.asarray(lat)
        self.kind = np.asarray(kind)
        self.A = self.lat.shape[0]
        self.directed, self.complete, self.prefer_direct = directed, complete, prefer_direct
        self.adjacent = adjacent
        self.self_loop_rule = self_loop_rule
        self.self_lat = None if self_lat is None else np.asarray(self_lat)
        self.self_rel = None
        self.self_kind = None if self_kind is None else np.asarray(self_kind)
        self.self_claimed = set()  # self pairs cached by the self-path rule (self_loop_rule)
        self.cache = {}          # (s, t) -> latency of the stored Path
        self.min_latency = 0.0   # topology.c minimumPathLatency
        self.upcalls = []        # every value handed to worker_updateMinTimeJump
        self.dijkstra_runs = 0
        self.self_paths = 0

    # ---------------------------------------------------------------- :1284-1386
    def _from_cache(self, s, t):
        return (s, t) if (s, t) in self.cache else None

    def _should_store(self, is_direct, s, t):
        if (s, t) in self.cache or (t, s) in self.cache:
            return False
        if self.complete and not is_direct:
            return False
        if self.prefer_direct and not is_direct and self.adjacent(s, t):
            return False
        return True

    def _store(self, is_direct, s, t, via_self=False):
        if not self._should_store(is_direct, s, t):
            return
        latency = float(self.self_lat[s] if via_self else self.lat[s, t])
        self.cache[(s, t)] = latency
        if via_self:
            self.self_claimed.add(s)
        if self.min_latency == 0 or latency < self.min_latency:
            self.min_latency = latency
            self.upcalls.append(latency)

    # ---------------------------------------------------------------- miss branches
    # each returns the reference's `success`
    def _lookup_direct(self, s, t):  # :1877-1927 (get_eid fails without an edge)
        if not self.adjacent(s, t):
            return False
        self._store(True, s, t)
        return True

    def _self_path(self, s):  # :1545-1653 (no incident edge: no path)
        self.self_paths += 1
        k = self.self_kind[s] if self.self_loop_rule else self.kind[s, s]
        if k == 0:
            return False
        self._store(False, s, s, via_self=self.self_loop_rule)
        return True

    def _compute_source_paths(self, s, t):  # :1655-1875
        if s == t:
            return self._self_path(s)
        self.dijkstra_runs += 1
        ok = True
        for position in range(self.A):  # the unique attached targets
            if position == s:
                if not self.self_loop_rule:
                    continue  # igraph's [] for the source: nothing stored (:1815)
                if self.kind[s, s] == 0:
                    ok = False  # [s] without a self-loop: get_eid fails (:1490-1495), the run is FALSE
                    continue
            if self.kind[s, position] == 0:  # igraph returns an empty path: nothing stored
                continue
            self._store(False, s, position)
        return ok

    # ---------------------------------------------------------------- :1969-2051
    def get_path_entry(self, s, t):
        """the (row, column) of the cached Path the query (s, t) returns, or None"""
        path = self._from_cache(s, t)
        if path is None and not self.directed:
            path = self._from_cache(t, s)
        if path is None:
            if self.complete or (self.prefer_direct and self.adjacent(s, t)):
                success = self._lookup_direct(s, t)
            else:
                success = self._compute_source_paths(s, t)
            if success:  # :2033-2038, directed or not
                path = self._from_cache(s, t) or self._from_cache(t, s)
        return path


def entry_value(model, path, lat, rel):
    """(latency, reliability) of the cached Path `path` = (row, column): the matrices' entry,
    or the self-path rule's value for a self pair that rule cached"""
    si, sj = path
    if si == sj and si in model.self_claimed:
        return float(model.self_lat[si]), float(model.self_rel[si])
    return float(lat[si, sj]), float(rel[si, sj])


def adjacency_of(g, attached=None):
    """adjacent(i, j) over attached indices of a synth graph (edge list g.src -> g.dst)"""
    att = list(g.attached if attached is None else attached)
    pairs = set()
    for a, b in zip(np.asarray(g.src).tolist(), np.asarray(g.dst).tolist()):
        pairs.add((a, b))
        if not g.directed:
            pairs.add((b, a))
    return lambda i, j: (att[i], att[j]) in pairs
