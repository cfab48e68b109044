#!/usr/bin/env python3
"""Drop-in shim rates, through the C harness tests/c/topo_harness.c
linked against libshadowtopo_hip as Shadow links it:
  * GraphML ingest + validation and 5e4 host attaches on the C5 graph (8.7e5 vertices)
    with IP-prefix, country/type and no hints (CPU only: no query, no GPU);
  * with --queries: per-call cost of the per-packet lookups (worker.c:267-279 sequence)
    under 1 and 8 threads on the C4 graph (1e4 hosts; needs the GPU for the one-shot build).
The graphs carry synthetic vertex attributes (ip, countrycode, type) so every hint kind has
candidates.  Writes one JSON object per run to stdout."""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def graphml_with_attrs(g, path):
    from shadow_amd import synth
    n = g.n
    ips = [f"10.{(v * 7) & 255}.{(v * 13) & 255}.{(v * 29) & 255}" for v in range(n)]
    cc = [("US", "DE", "FR", "BR", "JP")[v % 5] for v in range(n)]
    ty = [("client", "relay", "server")[v % 3] for v in range(n)]
    extra = {"ip": ("x1", "string", ips), "countrycode": ("x2", "string", cc), "type": ("x3", "string", ty)}
    with open(path, "w") as f:
        f.write(synth.to_graphml(g, extra_vattr=extra))


def build_harness(out_dir):
    from shadow_amd import engine as E
    lib_dir = os.path.dirname(E.LIB_PATH)
    exe = os.path.join(out_dir, "topo_harness")
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "topo_harness.c"), "-o", exe, "-L", lib_dir,
                    "-lshadowtopo_hip", f"-Wl,-rpath,{lib_dir}"], check=True)
    return exe


def run(exe, *args, warm=False):
    env = dict(os.environ, TOPO_HARNESS_WARM="1" if warm else "0")
    out = subprocess.run([exe] + [str(a) for a in args], check=True, capture_output=True, text=True, timeout=1800,
                         env=env)
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", action="store_true", help="also time per-packet lookups (GPU build)")
    ap.add_argument("--hosts", type=int, default=50_000)
    args = ap.parse_args()
    from shadow_amd import synth
    with tempfile.TemporaryDirectory() as tmp:
        exe = build_harness(tmp)
        if not args.queries:
            g = synth.chung_lu()
            path = os.path.join(tmp, "c5.graphml")
            graphml_with_attrs(g, path)
            for mode, name in ((0, "no hint"), (1, "country + type hints"), (2, "IP-prefix hints")):
                r = run(exe, path, args.hosts, 1, 0, mode)
                r.update({"graph": "C5", "hint_mode": name})
                print(json.dumps(r), flush=True)
        else:
            g = synth.barabasi_albert()
            path = os.path.join(tmp, "c4.graphml")
            graphml_with_attrs(g, path)
            # cold: the timed pass includes the emulated cache's first misses (one replayed
            # Dijkstra store loop per source); warm: an untimed pass first, then hits
            for warm in (False, True):
                for threads in (1, 8):
                    r = run(exe, path, 10_000, threads, 200_000, 0, warm=warm)
                    r.update({"graph": "C4", "hint_mode": "no hint"})
                    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
