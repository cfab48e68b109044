#!/usr/bin/env python3
"""A/B of k_walk's targets per wave (OPT_WALK_TPW) on C4L (the north-star graph with vertex
loss on 30 % of the vertices): compose + walk kernel time per build, the same rows each time."""
import hashlib
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402

g0 = synth.barabasi_albert(V=100_000, A=10_000)
out = {}
for name, g in (("C4", g0), ("C4L", synth.with_vertex_loss(g0))):
    eng = E.Engine.from_synth(g)
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_TIMING, 1)
    A = len(g.attached)
    dev = torch.device("cuda:0")
    lat = torch.empty((A, A), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    hops = torch.empty((A, A), dtype=torch.int32, device=dev)
    for tpw in ((2,) if name == "C4" else (1, 2, 3, 4, 1, 2)):
        eng.set_option(E.OPT_WALK_TPW, tpw)
        eng.compute_rows_device(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr())
        eng.reset_stats()
        t0 = time.perf_counter()
        for _ in range(3):
            eng.compute_rows_device(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr())
        torch.cuda.synchronize()
        st = eng.stats()
        h = hashlib.sha1(rel.cpu().numpy().tobytes()).hexdigest()[:12]
        rec = {"tpw": tpw, "compose_kernel_ms": st["compose_kernel_ms"] / 3, "ms": (time.perf_counter() - t0) / 3 * 1e3,
               "walk_targets": st["walk_targets"], "rel_sha": h}
        print(name, json.dumps(rec), flush=True)
        out.setdefault(name, []).append(rec)
    eng.close()
print(json.dumps(out))
