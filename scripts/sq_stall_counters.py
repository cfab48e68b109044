#!/usr/bin/env python3
"""Stall breakdown of one kernel from rocprofv3 --pmc passes (one directory per pass): every
counter summed over the last N dispatches whose name matches KERNEL_RE, then the ratios that
say where a wave's cycles go.  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count
quad-cycles (MI355X_MICROARCH.md), so only their ratios are used.
usage: sq_stall_counters.py KERNEL_RE N DIR [DIR ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    kre, n, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    tot = defaultdict(float)
    npass = defaultdict(int)  # passes that collected each counter (SQ_WAVE_CYCLES rides in every one)
    for d in dirs:
        per = defaultdict(lambda: defaultdict(float))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if re.search(kre, row.get("Kernel_Name", "")):
                    per[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        ks = sorted(per)[-n:]
        seen = set()
        for k in ks:
            for c, v in per[k].items():
                tot[c] += v
                seen.add(c)
        for c in seen:
            npass[c] += 1
        print(f"{d}: {len(ks)} dispatches")
    for c in tot:
        tot[c] /= max(1, npass[c])  # a counter collected by several passes: their mean
    for c in sorted(tot):
        print(f"  {c:28s} {tot[c]:.4g}")
    wc = tot.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
            if c in tot:
                print(f"  {c} / SQ_WAVE_CYCLES = {tot[c] / wc:.3f}")
    if tot.get("SQ_INSTS_LDS") and tot.get("SQ_LDS_BANK_CONFLICT") is not None:
        print(f"  LDS bank conflict cycles per LDS instruction = {tot['SQ_LDS_BANK_CONFLICT'] / tot['SQ_INSTS_LDS']:.3f}")


if __name__ == "__main__":
    main()
