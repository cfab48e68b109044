#!/usr/bin/env python3
"""Timing experiment: sparse rounds with D and P only (OPT 30, results invalid) against the
full tree-fold rounds, C4 and C5, rows left on the device; visits / rounds from OPT_PROFILE."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402

cfgs = sys.argv[1:] or ["C4"]
for cfg in cfgs:
    g = synth.barabasi_albert(V=100_000, A=10_000) if cfg == "C4" else synth.chung_lu(V=1_000_000, A=50_000)
    eng = E.Engine.from_synth(g)
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_TIMING, 1)
    A = len(g.attached)
    R = A if cfg == "C4" else 12_000  # C5: a 12 000-row share (one batch group)
    dev = torch.device("cuda:0")
    lat = torch.empty((R, A), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    hops = torch.empty((R, A), dtype=torch.int32, device=dev)
    for rep in range(2):
        for lean in (0, 1):
            eng.set_option(30, lean)
            for prof in (0, 1):
                eng.set_option(E.OPT_PROFILE, prof)
                eng.compute_rows_device(0, R, lat.data_ptr(), rel.data_ptr(), hops.data_ptr())
                torch.cuda.synchronize()
                eng.reset_stats()
                t0 = time.perf_counter()
                n = 2 if prof == 0 else 1
                for _ in range(n):
                    eng.compute_rows_device(0, R, lat.data_ptr(), rel.data_ptr(), hops.data_ptr())
                torch.cuda.synchronize()
                st = eng.stats()
                print(cfg, json.dumps({"lean": lean, "profile": prof, "ms": (time.perf_counter() - t0) / n * 1e3,
                                       "relax_ms": st["relax_ms"] / n, "rounds": st["rounds"] / n,
                                       "visits": st["visits"] / n, "changes": st["changes"] / n,
                                       "groups": st["groups"] / n}), flush=True)
    eng.close()
