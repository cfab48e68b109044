import ctypes, sys, time
import numpy as np
sys.path.insert(0, '/root/repo')
from shadow_amd import engine as E
E.LIB_PATH = sys.argv[1]
from shadow_amd import synth
g = synth.geometric_complete_ish(V=10_000, A=1_000)
eng = E.Engine.from_synth(g)
eng.set_attached(g.attached)
for _ in range(2):
    t = time.time(); eng.compute_rows(0, 1000); print("step s", time.time() - t, flush=True)
L = ctypes.CDLL(E.LIB_PATH)
n = (1 << 15) * 4
buf = np.zeros(n, np.int64)
assert L.shadowtopo_exp_dump(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n)) == 0
r = buf.reshape(-1, 4)
used = r[:, 3] > 0
r = r[used]
nblk = len(r) // 4
print("waves", len(r), "blocks", nblk)
tail, dr, ps, cyc = r[:, 0], r[:, 1], r[:, 2], r[:, 3] / 100.0
print("pairs/wave mean %.0f max %d  drains mean %.1f max %d  pass/drain %.3f" % (tail.mean(), tail.max(), dr.mean(), dr.max(), ps.sum() / dr.sum()))
print("wave time us: mean %.1f p50 %.1f p90 %.1f max %.1f" % (cyc.mean(), np.median(cyc), np.percentile(cyc, 90), cyc.max()))
print("us per drain: %.3f" % (cyc.sum() / dr.sum()))
bt = cyc.reshape(-1, 4)
print("block time (max over waves) mean %.1f; waves mean/blockmax %.2f" % (bt.max(1).mean(), (bt.mean(1) / bt.max(1)).mean()))
pw = tail.reshape(-1, 4)
print("pairs imbalance within block mean(mean/max) %.2f" % (pw.mean(1) / np.maximum(pw.max(1), 1)).mean())
# per batch pair totals (block L: q=L>>3, b=q%nb)
