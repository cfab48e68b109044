#!/bin/bash
# C4 with fewer batches in flight (groups whose state fits the Infinity Cache): one bench line each
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
for nb in 0 64 32 16 8 4; do
  timeout -k 10 300 python3 -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate --no-fresh --batches $nb > $O/c4_nb$nb.json 2> $O/c4_nb$nb.err || { echo "nb $nb failed"; tail -5 $O/c4_nb$nb.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c4_nb$nb.json')); e=d['engine']; print('batches $nb', round(d['ms_per_step'],1), 'ms; rounds/step', e['rounds_per_step'], 'groups', e.get('groups_per_step'), 'relax', round(e['relax_ms_per_step'],1))"
done
