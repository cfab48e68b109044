#!/usr/bin/env python3
"""Warm / cold per-packet lookup rates of two builds of the drop-in on ONE box (verdict r03
item 6): the current libshadowtopo_hip against the r02k build (commit 932dcde, built from
that commit's own sources into tools/abshim/r02k/), one harness (tests/c/topo_harness.c,
compiled against each build's own headers), C4 graph,
10^4 hosts, 8 threads and 1 thread, runs interleaved.  One JSON object per run."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from shim_rates import graphml_with_attrs, run  # noqa: E402


def build(src, lib_dir, inc, exe):
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-pthread", "-I", inc, src, "-o", exe, "-L", lib_dir,
                    "-lshadowtopo_hip", f"-Wl,-rpath,{lib_dir}"], check=True)
    return exe


def main():
    from shadow_amd import engine as E
    from shadow_amd import synth
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    with tempfile.TemporaryDirectory() as tmp:
        inc = os.path.join(ROOT, "include")
        builds = {
            "current": build(os.path.join(ROOT, "tests", "c", "topo_harness.c"), os.path.dirname(E.LIB_PATH), inc,
                             os.path.join(tmp, "h_cur")),
            # the same (current) harness, against r02k's headers and library: its warm pass
            # completes before the timed pass on every build
            "r02k": build(os.path.join(ROOT, "tests", "c", "topo_harness.c"),
                          os.path.join(ROOT, "tools", "abshim", "r02k"),
                          os.path.join(ROOT, "tools", "abshim", "r02k", "include"), os.path.join(tmp, "h_r02k")),
        }
        g = synth.barabasi_albert()
        path = os.path.join(tmp, "c4.graphml")
        graphml_with_attrs(g, path)
        for rep in range(reps):
            for name, exe in builds.items():
                for warm in (True, False):
                    for threads in (8, 1):
                        r = run(exe, path, 10_000, threads, 200_000, 0, warm=warm)
                        r.update({"build": name, "rep": rep})
                        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
