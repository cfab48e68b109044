#!/bin/bash
# r04 round check (suite, smoke, default bench, C3/C4/C5 lines) + lookup A/B, 4 interleaved reps
set -o pipefail
bash scripts/gpu_check.sh r04i C3 C4 C5 || exit 1
O=gpurun_out/r04i
timeout -k 10 900 python -u scripts/shim_ab.py 4 > $O/shim_ab.jsonl 2> $O/shim_ab.err || { tail $O/shim_ab.err; exit 1; }
python3 - <<'PY'
import json, statistics as S, collections
r = collections.defaultdict(list)
for l in open('gpurun_out/r04i/shim_ab.jsonl'):
    d = json.loads(l); r[(d['build'], 'warm' if d['warm'] else 'cold', d['threads'])].append(d['ns_per_call_per_thread'])
for k in sorted(r): print(k, 'median', round(S.median(r[k]), 1), 'all', [round(x) for x in r[k]])
PY
