#!/usr/bin/env python3
"""Step A/B on one engine: options given as NAME=v1,v2,... (engine OPT_ names); every
combination timed for `steps` builds, the whole set repeated `reps` times interleaved.
usage: _exp/c2_ab.py [--config C2|C3|C4|C5] STEPS REPS OPT=a,b [OPT=c,d ...]"""
import itertools
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402

args = sys.argv[1:]
cfg = "C2"
if args[0] == "--config":
    cfg, args = args[1], args[2:]
steps, reps = int(args[0]), int(args[1])
axes = []
for a in args[2:]:
    k, v = a.split("=")
    axes.append([(k, int(x)) for x in v.split(",")])
g = {"C2": lambda: synth.geometric_complete_ish(V=10_000, A=1_000), "C3": lambda: synth.knn_geographic(V=7_000),
     "C4": lambda: synth.barabasi_albert(V=100_000, A=10_000),
     "C5": lambda: synth.chung_lu(V=1_000_000, A=50_000)}[cfg]()
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
                                        "delta_ms": round(st["delta_ms"] / steps, 4), "relax_ms": round(st["relax_ms"] / steps, 3),
                                        "compose_kernel_ms": round(st["compose_kernel_ms"] / steps, 3),
                                        "rounds": st["rounds"] / steps, "groups": st["groups"] / steps})
        print(key, res[key][-1], flush=True)
print(json.dumps(res))
