"""Python mirror of Shadow's topology API (include/topology_hip.h) over ctypes.

Same names and error behaviour as /root/reference/src/main/routing/topology.h:17-28:
``Topology.new(path)`` returns None on a graph that fails validation, the getters
return -1.0 for an unroutable pair, ``isRoutable`` is ``getLatency > -1``.  Address and
Random are the library's standalone stand-ins (shadow_hooks.c); inside Shadow the real
objects are passed by the C caller instead.
"""
from __future__ import annotations

import ctypes
import socket
import struct

import numpy as np

from . import engine as _engine

TOPOLOGY_SYMBOLS = (
    "topology_new", "topology_free", "topology_attach", "topology_detach", "topology_isRoutable",
    "topology_getLatency", "topology_getReliability", "topology_incrementPathPacketCounter",
)
EXT_SYMBOLS = (
    "topology_hip_set_device", "topology_hip_set_devices", "topology_hip_set_self_rule", "topology_hip_prepare", "topology_hip_get_info",
    "topology_hip_attached", "topology_hip_vertex_of_ip", "topology_hip_vertex_of_id", "topology_hip_packet_count",
    "topology_hip_cached_cell", "topology_hip_edges", "shadowtopo_address_new", "shadowtopo_address_free", "shadowtopo_random_new",
    "shadowtopo_random_free", "shadowtopo_last_min_time_jump", "shadowtopo_min_time_jump_calls",
    "shadowtopo_set_log_level",
)


class Info(ctypes.Structure):
    _fields_ = [
        ("n_vertices", ctypes.c_int32), ("n_edges", ctypes.c_int64), ("is_directed", ctypes.c_int32),
        ("is_complete", ctypes.c_int32), ("is_connected", ctypes.c_int32), ("cluster_count", ctypes.c_int32),
        ("prefers_direct_paths", ctypes.c_int32), ("n_attached", ctypes.c_int32), ("computed_for", ctypes.c_int32),
        ("device", ctypes.c_int32), ("min_path_latency", ctypes.c_double), ("compute_seconds", ctypes.c_double),
        ("compute_count", ctypes.c_int64), ("n_devices", ctypes.c_int32), ("compute_failed", ctypes.c_int32),
        ("dijkstra_runs", ctypes.c_int64), ("self_path_count", ctypes.c_int64), ("cached_paths", ctypes.c_int64),
        ("self_seconds", ctypes.c_double),
        ("ip_table_slots", ctypes.c_int64), ("ip_tables_retired", ctypes.c_int64), ("ip_retired_bytes", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_configured = False


def lib():
    global _configured
    L = _engine.lib()
    if not _configured:
        vp = ctypes.c_void_p
        cp = ctypes.c_char_p
        L.topology_new.restype = vp
        L.topology_new.argtypes = [cp]
        L.topology_free.argtypes = [vp]
        L.topology_attach.argtypes = [vp, vp, vp, cp, cp, cp, cp, cp, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]
        L.topology_detach.argtypes = [vp, vp]
        L.topology_isRoutable.restype = ctypes.c_int
        L.topology_isRoutable.argtypes = [vp, vp, vp]
        L.topology_getLatency.restype = ctypes.c_double
        L.topology_getLatency.argtypes = [vp, vp, vp]
        L.topology_getReliability.restype = ctypes.c_double
        L.topology_getReliability.argtypes = [vp, vp, vp]
        L.topology_incrementPathPacketCounter.argtypes = [vp, vp, vp]
        L.topology_hip_set_device.argtypes = [vp, ctypes.c_int32]
        L.topology_hip_set_devices.argtypes = [vp, vp, ctypes.c_int32]
        L.topology_hip_set_self_rule.argtypes = [vp, ctypes.c_int32]
        L.topology_hip_prepare.argtypes = [vp]
        L.topology_hip_get_info.argtypes = [vp, ctypes.POINTER(Info)]
        L.topology_hip_attached.restype = ctypes.c_int32
        L.topology_hip_attached.argtypes = [vp, vp, ctypes.c_int32]
        L.topology_hip_vertex_of_ip.restype = ctypes.c_int32
        L.topology_hip_vertex_of_ip.argtypes = [vp, ctypes.c_uint32]
        L.topology_hip_vertex_of_id.restype = ctypes.c_int32
        L.topology_hip_vertex_of_id.argtypes = [vp, cp]
        L.topology_hip_packet_count.restype = ctypes.c_uint64
        L.topology_hip_packet_count.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.topology_hip_cached_cell.restype = ctypes.c_int32
        L.topology_hip_cached_cell.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.topology_hip_edges.argtypes = [vp] + [ctypes.POINTER(vp)] * 5
        L.shadowtopo_address_new.restype = vp
        L.shadowtopo_address_new.argtypes = [cp, cp]
        L.shadowtopo_address_free.argtypes = [vp]
        L.shadowtopo_random_new.restype = vp
        L.shadowtopo_random_new.argtypes = [ctypes.c_uint32]
        L.shadowtopo_random_free.argtypes = [vp]
        L.shadowtopo_last_min_time_jump.restype = ctypes.c_double
        L.shadowtopo_min_time_jump_calls.restype = ctypes.c_long
        L.shadowtopo_set_log_level.argtypes = [ctypes.c_int]
        _configured = True
    return L


def _b(s):
    return None if s is None else s.encode()


def ip_to_network(ip: str) -> int:
    """in_addr_t (network order) as the host stores it in a uint32"""
    return struct.unpack("=I", socket.inet_aton(ip))[0]


class Address:
    """standalone stand-in for Shadow's Address (main/routing/address.c)"""

    def __init__(self, ip: str, name: str = "host"):
        self._h = lib().shadowtopo_address_new(_b(ip), _b(name))
        if not self._h:
            raise ValueError(f"bad IPv4 address {ip!r}")
        self.ip = ip
        self.name = name

    def __del__(self):
        if getattr(self, "_h", None):
            lib().shadowtopo_address_free(self._h)
            self._h = None


class Random:
    """standalone stand-in for Shadow's Random (main/utility/random.c, rand_r based)"""

    def __init__(self, seed: int):
        self._h = lib().shadowtopo_random_new(seed)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().shadowtopo_random_free(self._h)
            self._h = None


def set_log_level(level: int):
    lib().shadowtopo_set_log_level(level)


def last_min_time_jump() -> float:
    return float(lib().shadowtopo_last_min_time_jump())


def min_time_jump_calls() -> int:
    """how many upcalls the standalone worker_updateMinTimeJump has received (process-wide)"""
    return int(lib().shadowtopo_min_time_jump_calls())


class Topology:
    def __init__(self, handle):
        self._h = handle

    @classmethod
    def new(cls, graph_path: str):
        """topology_new: None when the GraphML fails to load or validate"""
        h = lib().topology_new(_b(graph_path))
        return cls(h) if h else None

    def free(self):
        if getattr(self, "_h", None):
            lib().topology_free(self._h)
            self._h = None

    def __del__(self):
        self.free()

    def attach(self, address: Address, random: Random, ipHint=None, citycodeHint=None, countrycodeHint=None,
               geocodeHint=None, typeHint=None):
        down, up = ctypes.c_uint64(0), ctypes.c_uint64(0)
        lib().topology_attach(self._h, address._h, random._h if random else None, _b(ipHint), _b(citycodeHint),
                              _b(countrycodeHint), _b(geocodeHint), _b(typeHint), ctypes.byref(down),
                              ctypes.byref(up))
        return down.value, up.value

    def detach(self, address: Address):
        lib().topology_detach(self._h, address._h)

    def isRoutable(self, src: Address, dst: Address) -> bool:
        return bool(lib().topology_isRoutable(self._h, src._h, dst._h))

    def getLatency(self, src: Address, dst: Address) -> float:
        return float(lib().topology_getLatency(self._h, src._h, dst._h))

    def getReliability(self, src: Address, dst: Address) -> float:
        return float(lib().topology_getReliability(self._h, src._h, dst._h))

    def incrementPathPacketCounter(self, src: Address, dst: Address):
        lib().topology_incrementPathPacketCounter(self._h, src._h, dst._h)

    # ---- extensions (topology_hip_ext.h)
    def set_device(self, device: int):
        return lib().topology_hip_set_device(self._h, device)

    def set_devices(self, devices):
        arr = np.ascontiguousarray(devices, np.int32)
        return lib().topology_hip_set_devices(self._h, arr.ctypes.data_as(ctypes.c_void_p), len(arr))

    def set_self_rule(self, dijkstra_loop: bool):
        return lib().topology_hip_set_self_rule(self._h, int(dijkstra_loop))

    def prepare(self):
        return lib().topology_hip_prepare(self._h)

    def info(self):
        inf = Info()
        lib().topology_hip_get_info(self._h, ctypes.byref(inf))
        return inf.as_dict()

    def attached(self):
        n = lib().topology_hip_attached(self._h, None, 0)
        out = np.empty(max(n, 1), np.int32)
        lib().topology_hip_attached(self._h, out.ctypes.data_as(ctypes.c_void_p), n)
        return out[:n]

    def vertex_of_ip(self, ip: str) -> int:
        return int(lib().topology_hip_vertex_of_ip(self._h, ip_to_network(ip)))

    def vertex_of_id(self, node_id: str) -> int:
        return int(lib().topology_hip_vertex_of_id(self._h, _b(node_id)))

    def packet_count(self, src_vertex: int, dst_vertex: int) -> int:
        return int(lib().topology_hip_packet_count(self._h, src_vertex, dst_vertex))

    def cached_cell(self, src_vertex: int, dst_vertex: int) -> int:
        """bit 0: (src, dst) cached; bit 1: (dst, src) cached; -1: not attached"""
        return int(lib().topology_hip_cached_cell(self._h, src_vertex, dst_vertex))

    def edges(self):
        """(src, dst, latency, packetloss, vertex_packetloss) numpy copies of the parsed graph"""
        ptrs = [ctypes.c_void_p() for _ in range(5)]
        lib().topology_hip_edges(self._h, *[ctypes.byref(p) for p in ptrs])
        inf = self.info()
        m, n = inf["n_edges"], inf["n_vertices"]

        def arr(p, ct, k):
            if k == 0:
                return np.empty(0, ct)
            cptr = ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(ct)))
            return np.ctypeslib.as_array(cptr, shape=(k,)).copy()
        return (arr(ptrs[0], np.int32, m), arr(ptrs[1], np.int32, m), arr(ptrs[2], np.float64, m),
                arr(ptrs[3], np.float64, m), arr(ptrs[4], np.float64, n))
