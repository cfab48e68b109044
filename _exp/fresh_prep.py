#!/usr/bin/env python3
"""Fresh-attach preparation of a sparse config (run with SHADOWTOPO_TRACE_PREP=1): two
seeded attached sets alternating, rows into HBM, the host prep per build."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
g = {"C4": lambda: synth.barabasi_albert(V=100_000, A=10_000),
     "C5": lambda: synth.chung_lu(V=1_000_000, A=50_000)}[cfg]()
A = len(g.attached)
other = np.sort(np.random.default_rng(13).choice(g.n, size=A, replace=False)).astype(np.int32)
eng = E.Engine.from_synth(g)
dev = torch.device("cuda:0")
rows = A if cfg == "C4" else 2048
lat = torch.empty((rows, A), dtype=torch.float64, device=dev)
rel = torch.empty_like(lat)
hops = torch.empty((rows, A), dtype=torch.int32, device=dev)
for i, att in enumerate([g.attached, other, g.attached, other]):
    eng.set_attached(att)
    eng.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.compute_rows_device(0, rows, lat.data_ptr(), rel.data_ptr(), hops.data_ptr())
    torch.cuda.synchronize()
    print(f"build {i}: {1e3 * (time.perf_counter() - t0):.1f} ms, attach prep {eng.stats()['attach_prep_ms']:.1f} ms",
          file=sys.stderr, flush=True)
