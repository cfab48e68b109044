#!/bin/bash
# SQ + FETCH counter passes for one bench config per kernel variant: gpu_sq_ab.sh TAG CFG "args1" "args2" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
CFG=$1; shift
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES"
i=0
for a in "$@"; do
  i=$((i+1))
  B="bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate $a"
  timeout -s KILL 240 rocprofv3 --pmc $P1 -d gpurun_out/sq_${TAG}_$i -o pmc --output-format csv -- python3 $B > /dev/null 2> gpurun_out/sq_${TAG}_$i.err || { echo "sq pass $i failed"; tail -5 gpurun_out/sq_${TAG}_$i.err; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/sqf_${TAG}_$i -o pmc --output-format csv -- python3 $B > /dev/null 2> gpurun_out/sqf_${TAG}_$i.err || { echo "fetch pass $i failed"; exit 1; }
  echo "== $a"
  python3 scripts/pmc_summary.py gpurun_out/sq_${TAG}_$i gpurun_out/sqf_${TAG}_$i | grep -A12 "== k_relax" | head -26
done
