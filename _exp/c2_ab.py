#!/usr/bin/env python3
"""C2 step A/B on one engine: options given as NAME=v1,v2,... (engine OPT_ names); every
combination timed for `steps` builds, the whole set repeated `reps` times interleaved.
usage: _exp/c2_ab.py STEPS REPS OPT=a,b [OPT=c,d ...]"""
import itertools
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402

steps, reps = int(sys.argv[1]), int(sys.argv[2])
axes = []
for a in sys.argv[3:]:
    k, v = a.split("=")
    axes.append([(k, int(x)) for x in v.split(",")])
g = synth.geometric_complete_ish(V=10_000, A=1_000)
eng = E.Engine.from_synth(g)
eng.set_attached(g.attached)
eng.set_option(E.OPT_TIMING, 1)
A = len(g.attached)
dev = torch.device("cuda:0")
lat = torch.empty((A, A), dtype=torch.float64, device=dev)
rel = torch.empty_like(lat)
hops = torch.empty((A, A), dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream


def step():
    eng.compute_rows_device(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=s)


res = {}
for r in range(reps):
    for combo in itertools.product(*axes):
        for k, v in combo:
            eng.set_option(getattr(E, "OPT_" + k), v)
        step()
        step()
        torch.cuda.synchronize()
        eng.reset_stats()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        st = eng.stats()
        key = " ".join(f"{k}={v}" for k, v in combo)
        res.setdefault(key, []).append({"ms": round(ms, 4), "sweep_ms": round(st["full_ms"] / max(1, st["full_sweeps"]), 4),
                                        "delta_ms": round(st["delta_ms"] / steps, 4)})
        print(key, res[key][-1], flush=True)
print(json.dumps(res))
