#!/bin/bash
# build.sh NAME [defines...]: engine variant library _exp/lib_NAME.so
set -e
cd /root/repo/_exp
N=$1; shift
D=""; for d in "$@"; do D="$D -D$d"; done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off $D -I ../include -I ../shadow_amd/csrc -c ${SRC:-../shadow_amd/csrc/engine.hip} -o engine_$N.o
/opt/rocm/bin/hipcc -shared -fPIC ../shadow_amd/_build/graphml.c.o ../shadow_amd/_build/topology_hip.c.o ../shadow_amd/_build/shadow_hooks.c.o ../shadow_amd/_build/numparse.cpp.o ../shadow_amd/_build/graph_build.hip.o engine_$N.o -o lib_$N.so -pthread
