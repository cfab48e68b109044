#!/usr/bin/env python3
"""Extended seeded parity sweep (one process): the generators of tests/test_fuzz_gpu.py over
seeds past the suite's fixed range, every engine matrix against the oracle bit for bit.
usage: _exp/fuzz_extended.py SMALL_FROM SMALL_TO BIG_FROM BIG_TO"""
import sys
import time
import traceback

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_fuzz_gpu as F  # noqa: E402
from paritylib import compare  # noqa: E402

a, b, c, d = (int(x) for x in sys.argv[1:5])
fails = []
t0 = time.time()
n = 0
for seed in range(a, b):
    g, layout, opts = F._case(seed)
    if layout == "csr" and opts.get("worklist") == 0:
        opts.pop("device_rounds", None)
    try:
        compare(g, layout=layout, **opts)
    except AssertionError:
        fails.append(("small", seed, layout, opts, traceback.format_exc(limit=1)))
    n += 1
    if n % 50 == 0:
        print(f"{n} cases, {len(fails)} failed, {time.time() - t0:.0f} s", flush=True)
for seed in range(c, d):
    g, opts = F._big_case(seed)
    try:
        compare(g, **opts)
    except AssertionError:
        fails.append(("big", seed, None, opts, traceback.format_exc(limit=1)))
    n += 1
    if n % 10 == 0:
        print(f"{n} cases, {len(fails)} failed, {time.time() - t0:.0f} s", flush=True)
print(f"done: {n} cases, {len(fails)} failed, {time.time() - t0:.0f} s")
for f in fails:
    print(f)
sys.exit(1 if fails else 0)
