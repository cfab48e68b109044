#!/usr/bin/env python3
"""HBM traffic per step of each relax-family kernel from separate rocprofv3 FETCH_SIZE and
WRITE_SIZE passes over one bench command (_exp/scripts/ab_counters.sh): every dispatch of a kernel
whose name matches the regex is summed and divided by the bench's warmup + timed steps (the
engine's one-batch landmark rounds, run once before them, are included: ~1/157 of a C4 step).
FETCH_SIZE is doubled (gfx950 counts half of wide reads, MI355X_MICROARCH.md), WRITE_SIZE taken
as is, both KiB.

usage: ab_counters.py FETCH_DIR WRITE_DIR STEPS KERNEL_RE [OUT_JSON]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def per_kernel(d, counter, kre):
    tot = defaultdict(float)
    n = defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if row["Counter_Name"] != counter or not re.search(kre, name):
                    continue
                key = name.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].replace("void ", "")
                tot[key] += float(row["Counter_Value"]) * 1024
                n[key] += 1
    return tot, n


def main():
    fdir, wdir, steps, kre = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f, nf = per_kernel(fdir, "FETCH_SIZE", kre)
    w, _ = per_kernel(wdir, "WRITE_SIZE", kre)
    out = {"steps_counted": steps, "kernels": {}}
    total = 0.0
    for k in sorted(set(f) | set(w)):
        b = 2 * f.get(k, 0.0) + w.get(k, 0.0)
        total += b
        out["kernels"][k] = {"fetch_bytes_per_step": 2 * f.get(k, 0.0) / steps,
                             "write_bytes_per_step": w.get(k, 0.0) / steps,
                             "dispatches_per_step": nf.get(k, 0) / steps}
    out["hbm_bytes_per_step"] = total / steps
    print(json.dumps(out))
    if len(sys.argv) > 5:
        json.dump(out, open(sys.argv[5], "w"), indent=1)


if __name__ == "__main__":
    main()
