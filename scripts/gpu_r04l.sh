#!/bin/bash
# device-driven vs host-driven rounds on C4 row shares (8-rank share = 20 batches in flight)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
for b in 20 40; do
  for d in 1 0; do
    timeout -k 10 300 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --batches $b --device-rounds $d > $O/c4_b${b}_d$d.json 2> $O/c4_b${b}_d$d.err || { tail $O/c4_b${b}_d$d.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c4_b${b}_d$d.json')); e=d['engine']; print('batches $b devrounds $d', round(d['ms_per_step'],2), 'relax', round(e['relax_ms_per_step'],2), 'rounds', e['rounds_per_step'], 'syncs', e['host_syncs_per_step'])"
  done
done
