"""r03 exploration: C4 matrix build time vs batches in flight / device-driven rounds, and
per-rank row shares (1/2, 1/4, 1/8 of the rows) on one GPU."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from shadow_amd import engine as E, synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
g = synth.CONFIGS[cfg](1.0)
A = len(g.attached)
dev = torch.device("cuda:0")
eng = E.Engine.from_synth(g, device=0)
eng.set_attached(g.attached)
eng.set_option(E.OPT_TIMING, 1)
lat = torch.empty((A, A), dtype=torch.float64, device=dev)
rel = torch.empty((A, A), dtype=torch.float64, device=dev)
hops = torch.empty((A, A), dtype=torch.int32, device=dev)

def run(r0, r1, reps=3):
    s = torch.cuda.current_stream(dev).cuda_stream
    eng.compute_rows_device(r0, r1, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=s)
    torch.cuda.synchronize()
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.compute_rows_device(r0, r1, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    st = eng.stats()
    return {"rows": r1 - r0, "ms": dt * 1e3, "rounds": st["rounds"] / reps, "relax_ms": st["relax_ms"] / reps,
            "launches": st["relax_launches"] / reps}

ref = None
for nb, devr in [(0, 1), (64, 1), (32, 1), (32, 2), (16, 2), (8, 2), (4, 2), (2, 2)]:
    eng.set_option(E.OPT_BATCHES_IN_FLIGHT, nb)
    eng.set_option(E.OPT_DEVICE_ROUNDS, devr)
    r = run(0, A)
    h = hops.cpu().numpy(); l = lat.cpu().numpy()
    if ref is None:
        ref = (h.copy(), l.copy())
    r.update({"nb": nb, "device_rounds": devr, "same": bool(np.array_equal(h, ref[0]) and np.array_equal(l.view(np.uint64), ref[1].view(np.uint64)))})
    print(json.dumps(r), flush=True)
eng.set_option(E.OPT_BATCHES_IN_FLIGHT, 0)
eng.set_option(E.OPT_DEVICE_ROUNDS, 1)
for W in (2, 4, 8):
    per = -(-A // W)
    for r in range(min(W, 2)):
        x = run(r * per, min(A, (r + 1) * per))
        x.update({"share_of": W, "rank": r})
        print(json.dumps(x), flush=True)
eng.close()
