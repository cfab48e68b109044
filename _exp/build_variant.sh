#!/bin/bash
# experiment builds of the engine (-DSHADOWTOPO_EXPERIMENTS: the A/B getenv knobs) with extra -D flags:
# _exp/lib/libshadowtopo_<name>.so
# (loaded by setting SHADOWTOPO_EXP_LIB; the product loads shadow_amd/_build only)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
SRC=${SRC:-shadow_amd/csrc}  # another engine source dir (e.g. a git-show of an older engine.hip) for A/B builds
mkdir -p _exp/lib/$name
for s in engine graph_build; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -I include -I shadow_amd/csrc -DSHADOWTOPO_EXPERIMENTS "$@" -c $SRC/$s.hip -o _exp/lib/$name/$s.o
done
/opt/rocm/bin/hipcc -shared -fPIC _exp/lib/$name/engine.o _exp/lib/$name/graph_build.o shadow_amd/_build/graphml.c.o shadow_amd/_build/topology_hip.c.o shadow_amd/_build/shadow_hooks.c.o shadow_amd/_build/numparse.cpp.o -o _exp/lib/libshadowtopo_$name.so -pthread
echo _exp/lib/libshadowtopo_$name.so
