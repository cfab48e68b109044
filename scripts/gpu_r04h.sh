#!/bin/bash
# W16 diagnosis: hit rows (OPT_PROFILE) and per-kernel times with the f32 and fp16 chunk loops
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
for w in 0 1; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --dense-w16 $w --profile-counts > $O/c2p_w$w.json 2> $O/c2p_w$w.err || { tail $O/c2p_w$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2p_w$w.json')); e=d['engine']; print('w16=$w', round(d['ms_per_step'],3), 'visits', e['visits_per_step'], 'changes', e['changes_per_step'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$w -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --dense-w16 $w > $O/kt$w.json 2> $O/kt$w.err || { tail $O/kt$w.err; exit 1; }
  f=$(find $O/kt$w -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_w$w.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_w$w.csv')):
    if 'dense_f' in r['Name'] or 'delta_s' in r['Name']: print(r['Name'][:90], r['Calls'], r['AverageNs'])"
done
rm -rf $O/kt0 $O/kt1
