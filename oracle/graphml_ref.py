"""TEST INFRASTRUCTURE ONLY -- independent GraphML reader used as a checker.

Restates the parts of igraph's GraphML reader (igraph_read_graph_graphml, called at
/root/reference/src/main/routing/topology.c:386) that the topology path depends on,
written with xml.etree so it shares no code with the product's streaming C reader
(shadow_amd/csrc/graphml.c):

* vertex index = order of first appearance of a node id (in <node> or as an <edge>
  endpoint), edge index = order of <edge> elements;
* the node id string becomes the string vertex attribute "id";
* <key attr.type> int/long/float/double -> numeric (float), boolean -> boolean,
  string -> string; a missing numeric value is the key's <default> or NaN, a missing
  string the <default> or "";
* <graph edgedefault="directed|undirected"> sets directedness.

Never imported by the product path.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

NUMERIC_TYPES = {"int", "long", "float", "double"}


def _local(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


@dataclass
class RefGraph:
    directed: bool
    n: int
    src: np.ndarray
    dst: np.ndarray
    vattr: dict = field(default_factory=dict)   # name -> (type, list|ndarray)
    eattr: dict = field(default_factory=dict)
    gattr: dict = field(default_factory=dict)
    ids: list = field(default_factory=list)

    def vnum(self, name):
        t, v = self.vattr.get(name, (None, None))
        return None if t != "numeric" else v

    def enum(self, name):
        t, v = self.eattr.get(name, (None, None))
        return None if t != "numeric" else v


def _parse_num(text: str | None, default: float) -> float:
    if text is None:
        return default
    s = text.strip()
    if not s:
        return default
    try:
        return float(s)
    except ValueError:
        return math.nan


def read_graphml(text: str) -> RefGraph:
    root = ET.fromstring(text)
    keys = {}
    for k in root:
        if _local(k.tag) != "key":
            continue
        kid = k.get("id")
        name = k.get("attr.name", kid)
        atype = k.get("attr.type", "string")
        dom = k.get("for", "all")
        default = None
        for ch in k:
            if _local(ch.tag) == "default":
                default = ch.text or ""
        kind = "numeric" if atype in NUMERIC_TYPES else ("boolean" if atype == "boolean" else "string")
        keys[kid] = (name, kind, dom, default)
    graph = None
    for ch in root:
        if _local(ch.tag) == "graph":
            graph = ch
            break
    if graph is None:
        raise ValueError("no <graph> element")
    directed = graph.get("edgedefault", "directed") == "directed"
    ids = {}
    order = []

    def vid(name):
        if name not in ids:
            ids[name] = len(order)
            order.append(name)
        return ids[name]

    vdata = {}
    edges = []
    edata = []
    gdata = {}
    for el in graph:
        tag = _local(el.tag)
        if tag == "node":
            v = vid(el.get("id"))
            d = vdata.setdefault(v, {})
            for dd in el:
                if _local(dd.tag) == "data":
                    d[dd.get("key")] = dd.text or ""
        elif tag == "edge":
            a = vid(el.get("source"))
            b = vid(el.get("target"))
            edges.append((a, b))
            d = {}
            for dd in el:
                if _local(dd.tag) == "data":
                    d[dd.get("key")] = dd.text or ""
            edata.append(d)
        elif tag == "data":
            gdata[el.get("key")] = el.text or ""
    n = len(order)
    m = len(edges)
    g = RefGraph(directed=directed, n=n,
                 src=np.array([e[0] for e in edges], dtype=np.int32),
                 dst=np.array([e[1] for e in edges], dtype=np.int32),
                 ids=list(order))
    g.vattr["id"] = ("string", list(order))
    for kid, (name, kind, dom, default) in keys.items():
        if dom in ("node", "all"):
            if kind == "numeric":
                dv = _parse_num(default, math.nan) if default is not None else math.nan
                arr = np.full(n, dv, dtype=np.float64)
                for v, d in vdata.items():
                    if kid in d:
                        arr[v] = _parse_num(d[kid], dv)
                g.vattr[name] = ("numeric", arr)
            else:
                dv = default if default is not None else ""
                lst = [dv] * n
                for v, d in vdata.items():
                    if kid in d:
                        lst[v] = d[kid]
                g.vattr[name] = (kind, lst)
        if dom in ("edge", "all"):
            if kind == "numeric":
                dv = _parse_num(default, math.nan) if default is not None else math.nan
                arr = np.full(m, dv, dtype=np.float64)
                for e, d in enumerate(edata):
                    if kid in d:
                        arr[e] = _parse_num(d[kid], dv)
                g.eattr[name] = ("numeric", arr)
            else:
                dv = default if default is not None else ""
                g.eattr[name] = (kind, [d.get(kid, dv) for d in edata])
        if dom in ("graph", "all"):
            if kind == "numeric":
                dv = _parse_num(default, math.nan)
                g.gattr[name] = (kind, _parse_num(gdata[kid], dv) if kid in gdata else dv)
            else:
                g.gattr[name] = (kind, gdata.get(kid, default if default is not None else ""))
    return g
