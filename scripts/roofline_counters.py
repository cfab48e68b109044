#!/usr/bin/env python3
"""Per-launch counters of the bench's dominant relax kernel(s) -> profiles/roofline_counters.json
(read by bench.py as roofline.traffic and roofline.valu).

Inputs are three separate rocprofv3 --pmc passes over the SAME bench command
(scripts/gpu_roofline.sh): FETCH_SIZE, WRITE_SIZE, and an SQ pass (SQ_INSTS_VALU,
SQ_WAVES, GRBM_GUI_ACTIVE).  Corrections, MI355X_MICROARCH.md (HBM section):
  * FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of wide
    coalesced reads, so it is doubled; WRITE_SIZE is taken as is.
  * SQ counters do not cover every wave of a dispatch: the launch's true wave count
    (Grid_Size / 64) over SQ_WAVES scales SQ_INSTS_VALU up to the whole dispatch.
Which dispatches: those of the kernels matching KERNEL_RE, in dispatch order, the last
(warmup + steps) x launches_per_step of them -- exactly the bench's warmup and timed steps
(the engine's first computation also runs one-batch landmark rounds of the same kernels,
earlier) -- summed and divided by their count: bytes per launch averaged over the step's
launches, the unit of bench.py's roofline.

A launch may be several dispatches (PER_LAUNCH: the pruned dense sweep runs as two kernels,
its chunk loop and its exact pass, both matched by KERNEL_RE): then the last n x PER_LAUNCH
dispatches are summed and divided by n.

usage: roofline_counters.py KEY KERNEL_RE BENCH_JSON FETCH_DIR WRITE_DIR SQ_DIR [PER_LAUNCH]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def dispatches(d, kre):
    """[(dispatch_id, {counter: value, '_grid', '_ns'})] of matching kernels, in order"""
    out = defaultdict(lambda: defaultdict(float))
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not re.search(kre, row.get("Kernel_Name", "")):
                    continue
                k = int(row["Dispatch_Id"])
                out[k][row["Counter_Name"]] += float(row["Counter_Value"])
                out[k]["_grid"] = float(row["Grid_Size"])
                out[k]["_ns"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    return [out[k] for k in sorted(out)]


def main():
    key, kre, bench_json, fdir, wdir, sdir = sys.argv[1:7]
    per = int(sys.argv[7]) if len(sys.argv) > 7 else 1
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    rf = bench["roofline"]
    n = int(round((bench["warmup"] + bench["steps"]) * rf["launches_per_step"]))
    # label-correcting rounds read values that other waves of the same round may already have
    # updated, so a step can converge a round earlier or later from one run to the next: each
    # pass averages over its own last dispatches (at most n; up to a tenth fewer is accepted)
    f, w, s = (dispatches(d, kre)[-n * per:] for d in (fdir, wdir, sdir))
    if min(len(f), len(w), len(s)) < per * max(1, n - max(2, n // 10)):
        raise SystemExit(f"expected {n * per} dispatches matching {kre}, found {len(f)}/{len(w)}/{len(s)}")
    lf, lw, ls = (len(x) / per for x in (f, w, s))  # launches covered by each pass
    fetch = sum(v["FETCH_SIZE"] for v in f) * 1024 * 2 / lf
    write = sum(v["WRITE_SIZE"] for v in w) * 1024 / lw
    valu = sum(v["SQ_INSTS_VALU"] * (v["_grid"] / 64.0) / v["SQ_WAVES"] for v in s if v.get("SQ_WAVES")) / ls
    ns = sum(v["_ns"] for v in s)
    clk = sum(v["GRBM_GUI_ACTIVE"] for v in s) / 8.0 / ns if ns else None  # GHz
    rec = {"kernel": rf["kernel"], "batches_per_launch": rf["batches_per_launch"],
           "hbm_bytes_per_launch": fetch + write, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "valu_insts_per_launch": valu, "effective_clock_ghz_profiled": clk,
           "dispatches": n * per, "dispatches_per_launch": per, "dispatches_per_pass": [len(f), len(w), len(s)],
           "profiled_avg_launch_ms": sum(v["_ns"] for v in f) / lf / 1e6,
           "source": f"rocprofv3 --pmc passes over the bench command of {os.path.basename(bench_json)}: "
                     f"FETCH_SIZE x1024 x2, WRITE_SIZE x1024, SQ_INSTS_VALU x (Grid_Size/64)/SQ_WAVES; the last "
                     f"{n * per} dispatches of kernels matching '{kre}' ({per} per launch)"}
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "roofline_counters.json")
    db = json.load(open(p)) if os.path.exists(p) else {}
    db[key] = rec
    with open(p, "w") as fh:
        json.dump(db, fh, indent=1, sort_keys=True)
    print(json.dumps({key: rec}))


if __name__ == "__main__":
    main()
