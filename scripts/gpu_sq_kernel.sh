#!/bin/bash
# SQ counter passes (each list one pass) over one bench command, summed per kernel
# usage: scripts/gpu_sq_kernel.sh TAG "bench args" "COUNTERS1" ["COUNTERS2" ...]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
i=0
for c in "$@"; do
  O=gpurun_out/sq_${TAG}_$i
  mkdir -p $O
  timeout -s KILL 200 rocprofv3 --pmc $c -d $O -o pmc --output-format csv -- python3 bench.py $ARGS --no-cpu-baseline --no-host-rate > $O/b.json 2> $O/b.err || { echo "pass $i failed"; tail -5 $O/b.err; exit 1; }
  i=$((i+1))
done
python3 scripts/pmc_summary.py gpurun_out/sq_${TAG}_* | head -60
