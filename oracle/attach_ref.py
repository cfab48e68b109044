"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of the reference's host->vertex
attachment (/root/reference/src/main/routing/topology.c:2094-2369) and of the rand_r
stream behind random_nextDouble (src/main/utility/random.c:32-43), used to check the C
shim's topology_attach.  Small graphs only.
"""
from __future__ import annotations

import ctypes
import socket
import struct

INADDR_NONE = 0xFFFFFFFF
INADDR_ANY = 0
INADDR_LOOPBACK = 0x7F000001  # host-order constant compared against network-order IPs (:2127)

_libc = ctypes.CDLL(None)
_libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
_libc.rand_r.restype = ctypes.c_int
RAND_MAX = 2147483647


class RandR:
    """random_nextDouble: rand_r(&seedState) / RAND_MAX"""

    def __init__(self, seed):
        self.state = ctypes.c_uint(seed)

    def next_double(self):
        return float(_libc.rand_r(ctypes.byref(self.state))) / float(RAND_MAX)


def string_to_ip(s):
    """address_stringToIP (address.c:145-152): inet_pton, network order as a host uint32"""
    try:
        return struct.unpack("=I", socket.inet_pton(socket.AF_INET, s))[0]
    except (OSError, TypeError):
        return INADDR_NONE


def _usable(ip):
    return ip not in (INADDR_NONE, INADDR_ANY, INADDR_LOOPBACK)


def _crnd(x):
    """C round(): half away from zero"""
    import math
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def find_attachment_vertex(vattr, n, rnd, ipHint=None, citycodeHint=None, countrycodeHint=None, geocodeHint=None,
                           typeHint=None):
    """vattr: dict name -> list of per-vertex strings ('' = absent)"""
    def get(name, v):
        vals = vattr.get(name)
        s = vals[v] if vals is not None else ""
        return s if s else None

    Q = {k: [] for k in ("ct", "c", "kt", "k", "gt", "g", "t", "all")}
    N = {k: 0 for k in Q}
    requested, req_ok, exact = 0, False, False
    if ipHint:
        ip = string_to_ip(ipHint)
        if _usable(ip):
            req_ok, requested = True, ip
    eq = lambda a, b: a is not None and b is not None and a.lower() == b.lower()  # noqa: E731
    for v in range(n):
        ipS, city, country, geo, typ = (get(a, v) for a in ("ip", "citycode", "countrycode", "geocode", "type"))
        cm, km, gm, tm = eq(city, citycodeHint), eq(country, countrycodeHint), eq(geo, geocodeHint), eq(typ, typeHint)
        vu, vip = False, INADDR_NONE
        if ipS is not None:
            x = string_to_ip(ipS)
            if _usable(x):
                vu, vip = True, x
        if req_ok and vu and vip == requested:
            if not exact:
                for k in Q:
                    Q[k] = []
            exact = True
            Q["all"].append(v)
            N["all"] += 1
        if exact:
            continue
        Q["all"].append(v)
        N["all"] += vu
        for key, cond in (("ct", cm and tm), ("c", cm), ("kt", km and tm), ("k", km), ("gt", gm and tm), ("g", gm),
                          ("t", tm)):
            if cond:
                Q[key].append(v)
                N[key] += vu
    pick = next((k for k in ("ct", "c", "kt", "k", "gt", "g", "t") if Q[k]), "all")
    lpm = (req_ok and N[pick] > 0) if pick != "all" else bool(ipHint) and N["all"] > 0
    cand = Q[pick]
    if lpm and not exact:
        best_match, best = 0, -1
        for v in cand:
            vip = string_to_ip(get("ip", v) or "")
            match = (~(vip ^ requested)) & 0xFFFFFFFF
            if match > best_match or best_match == 0:
                best_match, best = match, v
        return best
    r = rnd.next_double()
    return cand[_crnd((len(cand) - 1) * r)]
