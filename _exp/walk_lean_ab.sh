#!/bin/bash
# r05: lean-walk shapes on C4 and C5, C3 with and without lean rounds
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 300 python3 -u _exp/c2_ab.py --config C4 3 2 WALK_TPW=1,2,3,4 > $O/c4_walk_ab.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u _exp/c2_ab.py --config C3 10 2 CSR_LEAN=0,1 > $O/c3_lean_ab.txt 2>&1 || exit 1
grep -v amdgpu $O/c4_walk_ab.txt | head -8
grep -v amdgpu $O/c3_lean_ab.txt | head -4
