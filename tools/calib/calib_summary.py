#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration summary (tools/calib/calib_fetch.hip): per access
shape, the known bytes each kernel moves against what rocprofv3's counters report.

usage: calib_summary.py PLAIN_JSON FETCH_DIR WRITE_DIR [RDREQ_DIR] > profiles/<tag>_fetch_calibration.json
"""
import csv
import glob
import json
import os
import sys


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if not name.startswith("k_"):
                continue
            out.setdefault(name, {}).setdefault(r["Counter_Name"], 0.0)
            out[name][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def main():
    plain = json.load(open(sys.argv[1]))
    f, w = counters(sys.argv[2]), counters(sys.argv[3])
    rq = counters(sys.argv[4]) if len(sys.argv) > 4 else {}
    best = {}
    for k in plain["kernels"]:
        best[k["kernel"]] = min(best.get(k["kernel"], 1e30), k["ms"])
    shapes = []
    for k in plain["kernels"]:
        if k["rep"] != 0:
            continue
        n = k["kernel"]
        known = k["known_bytes"] + k["index_bytes"]  # the index reads are coalesced 4 B/lane streams
        fetch = f.get(n, {}).get("FETCH_SIZE", 0.0) * 1024
        write = w.get(n, {}).get("WRITE_SIZE", 0.0) * 1024
        rec = {"kernel": n, "dir": k["dir"], "known_bytes": k["known_bytes"], "index_bytes": k["index_bytes"],
               "FETCH_SIZE_bytes": fetch, "WRITE_SIZE_bytes": write,
               "best_ms": best[n], "known_GBps": k["known_bytes"] / best[n] / 1e6}
        if k["dir"] == "read":
            rec["fetch_over_known"] = fetch / known
            rec["correction"] = known / fetch if fetch else None
        else:
            rec["write_over_known"] = write / k["known_bytes"]
        if n in rq:
            rec["TCC_EA0_RDREQ"] = rq[n].get("TCC_EA0_RDREQ_sum")
            rec["TCC_EA0_RDREQ_32B"] = rq[n].get("TCC_EA0_RDREQ_32B_sum")
        shapes.append(rec)
    print(json.dumps({"source": "tools/calib/calib_fetch.hip, 4 Mi rows of a 2 GiB table (each row or word read once, "
                                "the Infinity Cache flushed by a 1 GiB fill before every kernel); FETCH_SIZE / "
                                "WRITE_SIZE in KiB x 1024, separate rocprofv3 --pmc passes",
                      "shapes": shapes}, indent=1))


if __name__ == "__main__":
    main()
