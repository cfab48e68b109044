#!/bin/bash
# ab.sh LIBNAME... : bench each variant, print ms/step and the two dense kernels' launch times
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 200 python -u _exp/run.py $PWD/_exp/lib_$v.so --steps 5 --warmup 1 --no-cpu-baseline --no-host-rate $EXTRA > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.err || { echo "$v failed"; tail -5 gpurun_out/exp_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/exp_$v.json')); r=d['roofline']
print('$v', round(d['ms_per_step'],3), 'full', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
