"""Build recipe for libshadowtopo_hip.so (gfx950) -- run on the CPU container; the
built .so travels to the GPU box in-tree (git-ignored, not gpurun-ignored)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libshadowtopo_hip.so")
ARCH = os.environ.get("SHADOWTOPO_ARCH", "gfx950")

HIP_SOURCES = ["engine.hip", "graph_build.hip"]
C_SOURCES = ["graphml.c", "topology_hip.c", "shadow_hooks.c"]  # C host shim
CXX_SOURCES = ["numparse.cpp"]  # the GraphML reader's number conversion (std::from_chars)


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build(verbose=False, force=False):
    os.makedirs(OUT, exist_ok=True)
    inc = os.path.join(ROOT, "include")
    hip_srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    c_srcs = [os.path.join(CSRC, s) for s in C_SOURCES if os.path.exists(os.path.join(CSRC, s))]
    cxx_srcs = [os.path.join(CSRC, s) for s in CXX_SOURCES]
    headers = [os.path.join(inc, h) for h in os.listdir(inc)] + [
        os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if not force and not _stale(LIB, hip_srcs + c_srcs + cxx_srcs + headers):
        return LIB
    objs = []
    for s in c_srcs:
        o = os.path.join(OUT, os.path.basename(s) + ".o")
        _run(["gcc", "-O2", "-fPIC", "-std=gnu11", "-Wall", "-Wextra", "-pthread", "-ffp-contract=off",
              "-I", inc, "-I", CSRC, "-c", s, "-o", o], verbose)
        objs.append(o)
    for s in cxx_srcs:
        o = os.path.join(OUT, os.path.basename(s) + ".o")
        _run(["g++", "-O2", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-ffp-contract=off", "-c", s, "-o", o], verbose)
        objs.append(o)
    hipcc = _hipcc()
    for s in hip_srcs:
        o = os.path.join(OUT, os.path.basename(s) + ".o")
        _run([hipcc, "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=off",
              "-I", inc, "-I", CSRC, "-c", s, "-o", o], verbose)
        objs.append(o)
    tmp = LIB + ".tmp"
    _run([hipcc, "-shared", "-fPIC"] + objs + ["-o", tmp, "-pthread"], verbose)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
