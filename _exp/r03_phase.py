"""r03 diagnostic: per-block phase times of the dense full sweep (k_relax_dense_f, pruned) on
C2, from the EXP_PHASE_TIME build (s_memrealtime stamps, 100 MHz): init (thresholds +
seed), chunk loop, exact f64 pass, epilogue; chunks visited and logged rows per block."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from shadow_amd import engine as E, synth

g = synth.geometric_complete_ish(V=10_000, A=1_000)
A = len(g.attached)
eng = E.Engine.from_synth(g, device=0)
eng.set_attached(g.attached)
dev = torch.device("cuda:0")
lat = torch.empty((A, A), dtype=torch.float64, device=dev)
rel = torch.empty_like(lat)
hops = torch.empty((A, A), dtype=torch.int32, device=dev)
for _ in range(4):
    eng.compute_rows_device(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
L = E.lib()
nb = 8 * ((16 * ((10_000 + 31) // 32) + 7) // 8)
buf = np.zeros((nb, 8), np.uint64)
n = L.shadowtopo_exp_phase(buf.ctypes.data_as(ctypes.c_void_p), nb)
ok = buf[:, 4] > 0
b = buf[ok].astype(np.int64)
t0 = b[:, 0].min()
init, loop, exact, epi = (b[:, i + 1] - b[:, i] for i in range(4))
tick_us = 0.01
def st(x):
    x = x * tick_us
    return {"mean": float(x.mean()), "p50": float(np.median(x)), "p90": float(np.percentile(x, 90)), "max": float(x.max())}
rec = {"blocks": int(ok.sum()), "span_us": float((b[:, 4].max() - t0) * tick_us),
       "init_us": st(init), "loop_us": st(loop), "exact_us": st(exact), "epilogue_us": st(epi),
       "block_us": st(b[:, 4] - b[:, 0]),
       "chunks_visited": {"mean": float(b[:, 5].mean()), "max": int(b[:, 5].max())},
       "logged_rows_wave0": {"mean": float(b[:, 6].mean()), "max": int(b[:, 6].max())},
       "loop_us_per_chunk": float((loop * tick_us).sum() / max(1, b[:, 5].sum())),
       "start_us_pctl": [float(np.percentile((b[:, 0] - t0) * tick_us, q)) for q in (0, 25, 50, 75, 100)],
       "per_xcc_blocks": np.bincount((b[:, 7] >> 32).astype(np.int64), minlength=8).tolist()}
print(json.dumps(rec, indent=1))
eng.close()
