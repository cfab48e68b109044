#!/usr/bin/env python3
"""Generates the committed golden fixtures (run in the build container only; the GPU box
never reads /root/reference).

Inputs copied as data (not code) from the reference:
  * resource/topology.graphml.xml.xz          -> c1_topology.graphml.xml.xz (the shipped
    183-vertex complete topology, config 1)
  * the <topology> CDATA graphs of resource/examples/shadow.config.xml and of every
    src/test/**/*.test.shadow.config.xml       -> ref_test_graphs.json (deduplicated)

Expected outputs:
  * c1_direct.npz: the 183 x 183 attached-pair matrix under the complete-graph direct rule
    (topology.c:2019-2021, 1877-1927), computed here straight from the GraphML edge
    attributes with a dict (independent of the oracle's get_eid code):
    lat = latency(edge), rel = (1-lv_s)*(1-lv_t)*(1-loss(edge)).
  * ref_test_graphs.json: the self pair of each 1-vertex test graph (direct rule on the
    self-loop), e.g. latency 50.0 / reliability 0.99 for the example config
    (resource/examples/shadow.config.xml:11-21).
  * synthetic_*.npz: oracle outputs on small incomplete graphs -- regression pins only;
    the SSSP branch is "parity unpinned" (no reference fixture, igraph absent).
"""
from __future__ import annotations

import glob
import json
import lzma
import os
import re
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference"


def direct_matrix(g):
    lat_e = g.enum("latency")
    loss_e = g.enum("packetloss")
    vl = g.vnum("packetloss")
    edge = {}
    for e in range(len(g.src)):
        key = (min(g.src[e], g.dst[e]), max(g.src[e], g.dst[e]))
        edge.setdefault(key, e)  # lowest edge id
    n = g.n
    lat = np.full((n, n), -1.0)
    rel = np.full((n, n), -1.0)
    for s in range(n):
        for t in range(n):
            e = edge.get((min(s, t), max(s, t)))
            if e is None:
                continue
            r = 1.0
            if vl is not None and not np.isnan(vl[s]):
                r *= (1.0 - vl[s])
            if vl is not None and not np.isnan(vl[t]):
                r *= (1.0 - vl[t])
            lat[s, t] = 0.0 + lat_e[e]
            rel[s, t] = r * (1.0 - loss_e[e])
    return lat, rel


def main():
    from oracle.graphml_ref import read_graphml
    # --- C1 shipped topology
    src = os.path.join(REF, "resource", "topology.graphml.xml.xz")
    dst = os.path.join(HERE, "c1_topology.graphml.xml.xz")
    shutil.copyfile(src, dst)
    g = read_graphml(lzma.open(dst, "rt").read())
    lat, rel = direct_matrix(g)
    np.savez_compressed(os.path.join(HERE, "c1_direct.npz"), lat=lat, rel=rel, n=g.n, m=len(g.src))
    print(f"c1: V={g.n} E={len(g.src)}")
    # --- 1-vertex test graphs embedded in configs
    cfgs = [os.path.join(REF, "resource", "examples", "shadow.config.xml")]
    cfgs += sorted(glob.glob(os.path.join(REF, "src", "test", "**", "*.xml"), recursive=True))
    graphs = {}
    for c in cfgs:
        txt = open(c).read()
        m = re.search(r"<topology><!\[CDATA\[(.*?)\]\]></topology>", txt, re.S)
        if not m:
            continue
        gx = m.group(1)
        if gx in graphs:
            graphs[gx]["sources"].append(os.path.relpath(c, REF))
            continue
        rg = read_graphml(gx)
        l, r = direct_matrix(rg)
        graphs[gx] = {"graphml": gx, "sources": [os.path.relpath(c, REF)], "n": rg.n,
                      "self_latency": float(l[0, 0]), "self_reliability": float(r[0, 0])}
    out = list(graphs.values())
    json.dump(out, open(os.path.join(HERE, "ref_test_graphs.json"), "w"), indent=1)
    print(f"ref test graphs: {len(out)} unique from {len(cfgs)} configs")
    # --- synthetic regression pins from the oracle
    from oracle import oracle as O
    from shadow_amd import synth
    cases = {
        "synthetic_sparse": synth.random_sparse(V=120, avg_deg=4, seed=101),
        "synthetic_ties": synth.integer_grid(rows=8, cols=8, seed=5),
        "synthetic_directed": synth.random_sparse(V=100, avg_deg=4, seed=102, directed=True),
    }
    for name, sg in cases.items():
        og = O.OracleGraph(sg.n, sg.src, sg.dst, sg.latency, sg.packetloss, sg.vertex_packetloss,
                           directed=sg.directed)
        l, r, h, k, _ = og.pair_rows(og.flags(), sg.attached)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), n=sg.n, src=sg.src, dst=sg.dst,
                            latency=sg.latency, packetloss=sg.packetloss, vloss=sg.vertex_packetloss,
                            attached=sg.attached, directed=sg.directed, lat=l, rel=r, hops=h, kind=k)
        print(name, sg.n, sg.m)


if __name__ == "__main__":
    main()
