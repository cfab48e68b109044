#!/bin/bash
# r03 session 30: landmark count of the locality orders (MDS input) vs C2 sweep / C4 / C3 step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z6
mkdir -p $O
for run in "C2 8" "C2 16" "C2 32" "C2 64" "C2 8" "C2 16" "C4 8" "C4 16" "C4 32" "C3 8" "C3 16" "C3 32"; do
  set -- $run
  SHADOWTOPO_LANDMARKS=$2 timeout -k 10 300 python -u bench.py --config $1 --steps 5 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $O/$1_$2.json 2> $O/$1_$2.err || { echo "$run failed"; tail $O/$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2.json')); e=d['engine']; print('$1 L=$2', round(d['ms_per_step'],3), 'dom', round(d['roofline']['avg_launch_ms'],3), 'order', round(e['cold_start_parts_ms']['order'],1), 'first', round(e['cold_start_parts_ms']['first_step'],1))"
done
