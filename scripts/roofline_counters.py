#!/usr/bin/env python3
"""Per-launch counters of the bench's dominant kernel -> profiles/roofline_counters.json
(read by bench.py as roofline.traffic and roofline.valu).

Inputs are three separate rocprofv3 --pmc passes over the SAME bench command
(scripts/gpu_roofline.sh): FETCH_SIZE, WRITE_SIZE, and an SQ pass (SQ_INSTS_VALU,
SQ_WAVES, GRBM_GUI_ACTIVE).  Corrections, MI355X_MICROARCH.md (HBM section):
  * FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of wide
    coalesced reads, so it is doubled; WRITE_SIZE is taken as is.
  * SQ counters do not cover every wave of a dispatch: the launch's true wave count
    (Grid_Size / 64) over SQ_WAVES scales SQ_INSTS_VALU up to the whole dispatch.
Only dispatches of the named kernel with the bench's launch shape are used (the largest
grid: the engine's first computation also runs small one-batch landmark launches of the
same kernel), averaged per launch.

usage: roofline_counters.py KEY KERNEL_SUBSTR BENCH_JSON FETCH_DIR WRITE_DIR SQ_DIR
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, kernel_sub):
    """{(file, dispatch): {counter: value, '_grid': threads}}"""
    out = defaultdict(lambda: defaultdict(float))
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub not in row.get("Kernel_Name", ""):
                    continue
                k = (f, row["Dispatch_Id"])
                out[k][row["Counter_Name"]] += float(row["Counter_Value"])
                out[k]["_grid"] = float(row["Grid_Size"])
                out[k]["_ns"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    if out:  # the bench's own launches: the largest grid
        big = max(v["_grid"] for v in out.values())
        out = {k: v for k, v in out.items() if v["_grid"] == big}
    return out


def mean(xs):
    xs = list(xs)
    return sum(xs) / len(xs) if xs else None


def main():
    key, kernel, bench_json, fdir, wdir, sdir = sys.argv[1:7]
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    f = per_dispatch(fdir, kernel)
    w = per_dispatch(wdir, kernel)
    s = per_dispatch(sdir, kernel)
    if not f or not w or not s:
        raise SystemExit(f"no dispatches of {kernel}")
    fetch = mean(v["FETCH_SIZE"] * 1024 * 2 for v in f.values())
    write = mean(v["WRITE_SIZE"] * 1024 for v in w.values())
    valu = mean(v["SQ_INSTS_VALU"] * (v["_grid"] / 64.0) / v["SQ_WAVES"] for v in s.values() if v.get("SQ_WAVES"))
    clk = mean(v["GRBM_GUI_ACTIVE"] / 8.0 / v["_ns"] for v in s.values() if v.get("_ns"))  # GHz
    rf = bench["roofline"]
    rec = {"kernel": rf["kernel"], "batches_per_launch": rf["batches_per_launch"],
           "hbm_bytes_per_launch": fetch + write, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "valu_insts_per_launch": valu, "effective_clock_ghz_profiled": clk,
           "dispatches": [len(f), len(w), len(s)],
           "profiled_avg_launch_ms": mean(v["_ns"] for v in f.values()) / 1e6,
           "source": f"rocprofv3 --pmc passes over `{bench.get('_cmd', 'bench.py')}`: FETCH_SIZE x1024 x2, "
                     f"WRITE_SIZE x1024, SQ_INSTS_VALU x (Grid_Size/64)/SQ_WAVES; kernel filter '{kernel}'"}
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "roofline_counters.json")
    db = json.load(open(p)) if os.path.exists(p) else {}
    db[key] = rec
    with open(p, "w") as fh:
        json.dump(db, fh, indent=1, sort_keys=True)
    print(json.dumps({key: rec}))


if __name__ == "__main__":
    main()
