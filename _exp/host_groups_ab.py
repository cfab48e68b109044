#!/usr/bin/env python3
"""Host-delivered builds (rows, hop counts and kinds into page-locked host memory, PCIe
included) over OPT_HOST_GROUPS.  usage: _exp/host_groups_ab.py CONFIG REPS G1,G2,..."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402

cfg, reps, groups = sys.argv[1], int(sys.argv[2]), [int(x) for x in sys.argv[3].split(",")]
g = {"C3": lambda: synth.knn_geographic(V=7_000), "C4": lambda: synth.barabasi_albert(V=100_000, A=10_000),
     "C2": lambda: synth.geometric_complete_ish(V=10_000, A=1_000)}[cfg]()
eng = E.Engine.from_synth(g)
eng.set_attached(g.attached)
A = len(g.attached)
outs = [E.pinned_empty((A, A), np.float64), E.pinned_empty((A, A), np.float64),
        E.pinned_empty((A, A), np.uint32), E.pinned_empty((A, A), np.uint8)]
for _ in range(2):
    for ng in groups:
        eng.set_option(E.OPT_HOST_GROUPS, ng)
        eng.compute_rows_into(0, A, *outs)
        eng.reset_stats()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.compute_rows_into(0, A, *outs)
            ts.append((time.perf_counter() - t0) * 1e3)
        st = eng.stats()
        print(f"{cfg} host groups {ng}: " + " ".join(f"{t:.1f}" for t in ts) + f" ms (groups per call {st['groups'] / reps:.0f})", flush=True)
