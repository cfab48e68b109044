#!/usr/bin/env python3
"""Per-step GPU timeline of a bench run from a rocprofv3 kernel trace (csv): for the last N
steps (each step starts at the kernel named by --first), the busy time (sum of kernel
durations), the span, and the idle gaps between consecutive kernels with what follows them."""
import csv, sys, argparse, glob
ap = argparse.ArgumentParser()
ap.add_argument("trace_dir")
ap.add_argument("--first", default="k_seed_dense_t")
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--span", default=None, help="also print, per step, the span from the first start to the last end "
                                              "of the kernels matching this regex (concurrent dispatches of one launch)")
a = ap.parse_args()
import re
f = glob.glob(a.trace_dir + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
sel = starts[-a.steps - 1:]  # boundaries of the last steps (the last one runs to the end)
for si in range(len(sel)):
    lo = sel[si]; hi = sel[si + 1] if si + 1 < len(sel) else len(rows)
    ks = rows[lo:hi]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks) / 1e3
    span = (int(ks[-1]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"])) / 1e3
    print(f"step {si}: {len(ks)} kernels, busy {busy:.1f} us, span {span:.1f} us")
    if a.span:
        m = [r for r in ks if re.search(a.span, r["Kernel_Name"])]
        if m:
            sp = (max(int(r["End_Timestamp"]) for r in m) - min(int(r["Start_Timestamp"]) for r in m)) / 1e3
            print(f"   span of {len(m)} dispatches matching {a.span!r}: {sp:.1f} us")
    for p, q in zip(ks, ks[1:]):
        gap = (int(q["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3
        dur = (int(q["End_Timestamp"]) - int(q["Start_Timestamp"])) / 1e3
        print(f"   gap {gap:8.1f} us  -> {q['Kernel_Name'][:70]} ({dur:.1f} us)")
