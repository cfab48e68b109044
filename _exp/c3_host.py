#!/usr/bin/env python3
"""C3 host-delivered build (pinned rows, PCIe included): with and without hop counts."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402

g = synth.knn_geographic(V=7_000)
eng = E.Engine.from_synth(g)
eng.set_attached(g.attached)
if len(sys.argv) > 1:
    eng.set_option(E.OPT_SPIN_US, int(sys.argv[1]))
A = len(g.attached)
outs = [E.pinned_empty((A, A), np.float64), E.pinned_empty((A, A), np.float64),
        E.pinned_empty((A, A), np.uint32), E.pinned_empty((A, A), np.uint8)]
for hops in (True, False, True, False):
    o = list(outs)
    if not hops:
        o[2] = None
    eng.compute_rows_into(0, A, *o)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        eng.compute_rows_into(0, A, *o)
        ts.append((time.perf_counter() - t0) * 1e3)
    st = eng.stats()
    print(f"hops={hops}: " + " ".join(f"{t:.2f}" for t in ts) + f" ms  groups={st['groups']}", flush=True)
