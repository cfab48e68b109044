import sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from shadow_amd import engine as E
if len(sys.argv) > 1: E.LIB_PATH = sys.argv[1]
from shadow_amd import synth
from paritylib import compare
g = synth.random_sparse(V=301, avg_deg=5, seed=1)
for prune in (0, 1):
    try:
        st = compare(g, layout="dense", dense_prune=prune); print("prune", prune, "ok", st["pruned_deltas"], st["delta_sweeps"], st["full_sweeps"])
    except AssertionError as e:
        print("prune", prune, "FAIL", str(e)[:150])
