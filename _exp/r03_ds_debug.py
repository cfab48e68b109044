"""debug: delta-stepping rounds -- failures per batch (r03x)"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from paritylib import oracle_matrix, engine_matrix
from shadow_amd import synth
g = synth.random_sparse(V=1100, avg_deg=4, seed=23)
lat_o, rel_o, hops_o, kind_o, _ = oracle_matrix(g)
for opts in [dict(batches_in_flight=1, delta_step=5000, device_rounds=0),
             dict(batches_in_flight=1, delta_step=5000, device_rounds=0, worklist=2),
             dict(batches_in_flight=1, delta_step=5000, device_rounds=0, prune_pendant=0, source_order=0),
             dict(batches_in_flight=1, delta_step=0, device_rounds=0)]:
    lat, rel, hops, kind, st = engine_matrix(g, **opts)
    bad = (lat.view(np.uint64) != lat_o.view(np.uint64))
    per = bad.reshape(-1)[: (bad.shape[0] // 64) * 64 * bad.shape[1]].reshape(-1, 64 * bad.shape[1]).sum(1)
    higher = int((lat > lat_o).sum()); lower = int((lat < lat_o).sum())
    print(opts, "mismatch", int(bad.sum()), "higher", higher, "lower", lower, "per batch", list(per), "rounds", st["rounds"], flush=True)
