#!/usr/bin/env python3
"""Sum rocprofv3 counter_collection.csv values per (kernel, counter) over the given dirs."""
import collections
import csv
import glob
import os
import sys

tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
kernels = sorted({k for k, _ in tot}, key=lambda k: -tot.get((k, "SQ_WAVE_CYCLES"), 0))
for k in kernels:
    print(f"== {k}  dispatches={len(disp[k])}")
    for (kk, c), v in sorted(tot.items()):
        if kk == k:
            print(f"   {c:24s} {v:.4g}")
