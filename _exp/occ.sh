#!/bin/bash
set -o pipefail
for occ in 0 6 5 4 3 0; do
  timeout -k 10 200 python -u _exp/run.py $PWD/_exp/lib_N4.so --steps 5 --warmup 1 --no-cpu-baseline --no-host-rate --dense-occ $occ > gpurun_out/occ_$occ.json 2> gpurun_out/occ_$occ.err || { echo "occ $occ failed"; tail -5 gpurun_out/occ_$occ.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/occ_$occ.json')); r=d['roofline']
print('occ $occ', round(d['ms_per_step'],3), 'full', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
