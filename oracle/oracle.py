"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the CPU restatement (topo_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline -- never as the product path.
See topo_oracle.c for the restated reference functions and their file:line citations.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libtopo_oracle.so")

OG_DIRECTED = 1
OG_COMPLETE = 2
OG_PREFER_DIRECT = 4
OG_SELF_DIJKSTRA_LOOP = 8

KIND_FAIL, KIND_DIRECT, KIND_SELF, KIND_DIJKSTRA = 0, 1, 2, 3

_lib = None

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.og_new.restype = ctypes.c_void_p
        L.og_new.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int, _i32p, _i32p, _f64p, _f64p, _f64p]
        L.og_free.argtypes = [ctypes.c_void_p]
        L.og_get_eid.restype = ctypes.c_int64
        L.og_get_eid.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        L.og_is_complete.restype = ctypes.c_int
        L.og_is_complete.argtypes = [ctypes.c_void_p]
        L.og_dijkstra.restype = ctypes.c_int64
        L.og_dijkstra.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                  _f64p, _i64p, ctypes.c_void_p]
        L.og_path.restype = ctypes.c_int32
        L.og_path.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _i64p, _i32p, ctypes.c_int32]
        L.og_pair_rows.restype = ctypes.c_int
        L.og_pair_rows.argtypes = [ctypes.c_void_p, ctypes.c_uint32, _i32p, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, _f64p, _f64p, _u32p, _u8p, ctypes.c_int]
        L.og_pair_rows_list.restype = ctypes.c_int
        L.og_pair_rows_list.argtypes = [ctypes.c_void_p, ctypes.c_uint32, _i32p, ctypes.c_int32, _i32p,
                                        ctypes.c_int32, _f64p, _f64p, _u32p, _u8p, ctypes.c_int]
        L.og_tie_vertices.argtypes = [ctypes.c_void_p, ctypes.c_int32, _f64p, _u8p]
        L.og_self_path.restype = ctypes.c_int
        L.og_self_path.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


class OracleGraph:
    """Graph in igraph edge order (src/dst as read from GraphML, before igraph's
    from=max/to=min normalisation of undirected edges)."""

    def __init__(self, n, src, dst, latency, packetloss, vertex_packetloss=None, directed=False):
        L = lib()
        self.n = int(n)
        self.m = len(src)
        self.directed = bool(directed)
        self.src = np.ascontiguousarray(src, dtype=np.int32)
        self.dst = np.ascontiguousarray(dst, dtype=np.int32)
        self.lat = np.ascontiguousarray(latency, dtype=np.float64)
        self.loss = np.ascontiguousarray(packetloss, dtype=np.float64)
        if vertex_packetloss is None:
            vertex_packetloss = np.full(self.n, np.nan)
        self.vloss = np.ascontiguousarray(vertex_packetloss, dtype=np.float64)
        self._h = L.og_new(self.n, self.m, int(self.directed), self.src, self.dst, self.lat, self.loss, self.vloss)
        if not self._h:
            raise MemoryError("og_new failed")

    def close(self):
        if getattr(self, "_h", None):
            lib().og_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def get_eid(self, a, b):
        return int(lib().og_get_eid(self._h, int(a), int(b)))

    def is_complete(self):
        return bool(lib().og_is_complete(self._h))

    def dijkstra(self, source, targets=None, want_order=False):
        dist = np.empty(self.n, np.float64)
        parent = np.empty(self.n, np.int64)
        order = np.empty(self.n, np.int32) if want_order else None
        if targets is not None:
            t = np.ascontiguousarray(targets, dtype=np.int32)
            tp, nt = t.ctypes.data_as(ctypes.c_void_p), len(t)
        else:
            t, tp, nt = None, None, 0
        npop = lib().og_dijkstra(self._h, int(source), tp, nt, dist, parent,
                                 order.ctypes.data_as(ctypes.c_void_p) if want_order else None)
        if want_order:
            return dist, parent, order[:npop]
        return dist, parent

    def path(self, source, node, parent):
        out = np.empty(self.n + 1, np.int32)
        k = lib().og_path(self._h, int(source), int(node), parent, out, self.n + 1)
        return out[:max(k, 0)]

    def self_path(self, v):
        lat, rel = ctypes.c_double(), ctypes.c_double()
        ok = lib().og_self_path(self._h, int(v), ctypes.byref(lat), ctypes.byref(rel))
        return (lat.value, rel.value) if ok else None

    def pair_rows(self, flags, attached, row_begin=0, row_end=None, nthreads=1):
        att = np.ascontiguousarray(attached, dtype=np.int32)
        A = len(att)
        if row_end is None:
            row_end = A
        R = row_end - row_begin
        lat = np.empty(R * A, np.float64)
        rel = np.empty(R * A, np.float64)
        hops = np.empty(R * A, np.uint32)
        kind = np.empty(R * A, np.uint8)
        fails = lib().og_pair_rows(self._h, int(flags), att, A, row_begin, row_end, lat, rel, hops, kind, nthreads)
        return (lat.reshape(R, A), rel.reshape(R, A), hops.reshape(R, A), kind.reshape(R, A), fails)

    def pair_rows_list(self, flags, attached, rows, nthreads=1):
        """pair_rows for an arbitrary list of source rows (output row q = rows[q])"""
        att = np.ascontiguousarray(attached, dtype=np.int32)
        rw = np.ascontiguousarray(rows, dtype=np.int32)
        A, R = len(att), len(rw)
        assert ((rw >= 0) & (rw < A)).all()
        lat = np.empty(R * A, np.float64)
        rel = np.empty(R * A, np.float64)
        hops = np.empty(R * A, np.uint32)
        kind = np.empty(R * A, np.uint8)
        fails = lib().og_pair_rows_list(self._h, int(flags), att, A, rw, R, lat, rel, hops, kind, nthreads)
        return (lat.reshape(R, A), rel.reshape(R, A), hops.reshape(R, A), kind.reshape(R, A), fails)

    def tie_vertices(self, source, dist):
        tie = np.empty(self.n, np.uint8)
        lib().og_tie_vertices(self._h, int(source), np.ascontiguousarray(dist), tie)
        return tie

    def flags(self, prefer_direct=False, self_dijkstra_loop=False):
        f = OG_DIRECTED if self.directed else 0
        if self.is_complete():
            f |= OG_COMPLETE
        if prefer_direct:
            f |= OG_PREFER_DIRECT
        if self_dijkstra_loop:
            f |= OG_SELF_DIJKSTRA_LOOP
        return f


def from_refgraph(g):
    """OracleGraph from graphml_ref.RefGraph (latency/packetloss edge attrs)."""
    lat = g.enum("latency")
    loss = g.enum("packetloss")
    vl = g.vnum("packetloss")
    return OracleGraph(g.n, g.src, g.dst, lat, loss, vl, directed=g.directed)
